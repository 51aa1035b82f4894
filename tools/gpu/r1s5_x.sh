set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
timeout -k 10 300 python -u -m pytest tests/test_backbone_ops_gpu.py -x -q --timeout 120 --timeout-method thread > gpurun_out/s5x_tests.log 2>&1 || { echo "tests failed"; tail -40 gpurun_out/s5x_tests.log; exit 1; }
tail -1 gpurun_out/s5x_tests.log
timeout -k 10 300 python -u bench.py --no-cpu-baseline > gpurun_out/s5x_bench.log 2>&1 || { tail -30 gpurun_out/s5x_bench.log; exit 1; }
tail -1 gpurun_out/s5x_bench.log | cut -c1-200
