set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
timeout -k 10 400 python -u -m pytest tests -x -q -m gpu --timeout 120 --timeout-method thread > gpurun_out/s2a_tests.log 2>&1 && \
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/s2a_smoke.log 2>&1 && \
timeout -k 10 500 python bench.py > gpurun_out/s2a_bench.json 2> gpurun_out/s2a_bench.err
