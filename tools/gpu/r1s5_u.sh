set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
timeout -k 10 300 python -u -m pytest tests/test_conv_gpu.py -x -q --timeout 120 --timeout-method thread > gpurun_out/s5u_tests.log 2>&1 || { echo "tests failed"; tail -40 gpurun_out/s5u_tests.log; exit 1; }
tail -1 gpurun_out/s5u_tests.log
timeout -k 10 300 python -u tools/conv_bench.py > gpurun_out/s5u_conv.log 2>&1 || { tail -20 gpurun_out/s5u_conv.log; exit 1; }
grep -v amdgpu.ids gpurun_out/s5u_conv.log | head -2
