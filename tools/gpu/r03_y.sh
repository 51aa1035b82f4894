# round 3, call y: the full GPU suite + smoke (as the driver runs them), then the default bench line
set -o pipefail
R=$GRAFT_REPO_ROOT
cd "$R" && mkdir -p gpurun_out && export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 200 --timeout-method thread > gpurun_out/tests_y.log 2>&1 && \
echo "[y] tests ok" && \
timeout -k 10 200 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke_y.log 2>&1 && echo "[y] smoke ok" && \
timeout -k 10 500 python -u bench.py > gpurun_out/bench_y.json 2> gpurun_out/bench_y.err && echo "[y] bench ok"
