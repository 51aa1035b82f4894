set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
timeout -k 10 300 python -u -m pytest tests/test_linear_gpu.py -x -q -m gpu --timeout 120 --timeout-method thread > gpurun_out/s2c_tests.log 2>&1; echo "tests rc=$?" >> gpurun_out/s2c_tests.log
timeout -k 10 300 python tools/gemm_x3_bench.py > gpurun_out/s2c_bench.log 2>&1
