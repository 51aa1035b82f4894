set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
for a in 0 8; do M2F_MSDA_ABLATE=$a timeout -k 10 120 python tools/msda_bench.py --bwd-only >> gpurun_out/s2p_bench.log 2>&1; done
M2F_MSDA_DETERMINISTIC=1 timeout -k 10 120 python tools/msda_bench.py --bwd-only >> gpurun_out/s2p_bench.log 2>&1
timeout -k 10 300 python -u -m pytest tests/test_msda_gpu.py -x -q -m gpu --timeout 120 --timeout-method thread > gpurun_out/s2p_tests.log 2>&1; echo "tests rc=$?" >> gpurun_out/s2p_tests.log
