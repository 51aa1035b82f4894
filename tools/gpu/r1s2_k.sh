set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
timeout -k 10 300 python -u -m pytest tests/test_msda_gpu.py -x -q -m gpu --timeout 120 --timeout-method thread > gpurun_out/s2k_tests.log 2>&1; echo "tests rc=$?" >> gpurun_out/s2k_tests.log
for bb in 1 0; do for h in 8 6; do
  M2F_MSDA_BBOX=$bb M2F_MSDA_HALO=$h timeout -k 10 120 python tools/msda_bench.py --bwd-only >> gpurun_out/s2k_bench.log 2>&1
done; done
M2F_MSDA_BBOX=0 M2F_MSDA_HALO=6 timeout -k 10 300 python -u -m pytest tests/test_msda_gpu.py -x -q -m gpu --timeout 120 --timeout-method thread > gpurun_out/s2k_tests0.log 2>&1; echo "tests rc=$?" >> gpurun_out/s2k_tests0.log
