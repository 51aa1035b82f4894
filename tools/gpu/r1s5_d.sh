set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
timeout -k 10 300 python -u -m pytest tests/test_conv_gpu.py -x -q --timeout 120 --timeout-method thread > gpurun_out/s5d_tests.log 2>&1 || { echo "tests failed"; tail -30 gpurun_out/s5d_tests.log; exit 1; }
tail -1 gpurun_out/s5d_tests.log
M2F_CONV3_WGRAD=x3 timeout -k 10 300 python -u tools/conv_bench.py > gpurun_out/s5d_conv.log 2>&1 || { tail -20 gpurun_out/s5d_conv.log; exit 1; }
grep -v amdgpu.ids gpurun_out/s5d_conv.log
M2F_CONV3_WGRAD=x3 timeout -k 10 300 python -u bench.py --no-cpu-baseline > gpurun_out/s5d_bench.log 2>&1 || { tail -30 gpurun_out/s5d_bench.log; exit 1; }
tail -1 gpurun_out/s5d_bench.log | cut -c1-200
