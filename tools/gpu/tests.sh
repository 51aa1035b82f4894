# The GPU test suite as the driver runs it, plus smoke() -> gpurun_out/tests_gpu.log
set -o pipefail
cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out && export TMPDIR=/tmp
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread 2>&1 | tee gpurun_out/tests_gpu.log | grep --line-buffered -E "FAIL|ERROR|passed|failed" && \
timeout -k 10 200 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')"
