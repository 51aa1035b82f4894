# final tree (+ wave combine): full GPU suite, smoke, default bench
set -o pipefail
cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out && export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r5an_tests.log 2>&1 || exit 1
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" >> gpurun_out/r5an_tests.log 2>&1 || exit 1
timeout -k 10 600 python3 bench.py > gpurun_out/r5an_bench.json 2> gpurun_out/r5an_bench.err
