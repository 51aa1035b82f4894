set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
timeout -k 10 300 python -u -m pytest tests/test_linear_gpu.py tests/test_modules_gpu.py -x -q --timeout 120 --timeout-method thread > gpurun_out/s5b_tests.log 2>&1 || { echo "targeted tests failed"; tail -30 gpurun_out/s5b_tests.log; exit 1; }
timeout -k 10 300 python -u bench.py --no-cpu-baseline > gpurun_out/s5b_bench.log 2>&1 || { tail -30 gpurun_out/s5b_bench.log; exit 1; }
M2F_RESIDUAL_FUSED=0 timeout -k 10 300 python -u bench.py --no-cpu-baseline > gpurun_out/s5b_bench_unfused.log 2>&1
tail -2 gpurun_out/s5b_tests.log; tail -1 gpurun_out/s5b_bench.log; tail -1 gpurun_out/s5b_bench_unfused.log
