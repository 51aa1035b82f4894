set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
timeout -k 10 300 python -u -m pytest tests/test_msda_gpu.py -x -q -m gpu --timeout 120 --timeout-method thread > gpurun_out/s2i_tests.log 2>&1; echo "tests rc=$?" >> gpurun_out/s2i_tests.log
for cfg in "16 512" "12 512" "8 512" "16 1024" "12 768"; do
  set -- $cfg
  M2F_MSDA_TILE=$1 M2F_MSDA_THREADS=$2 timeout -k 10 120 python tools/msda_bench.py --bwd-only >> gpurun_out/s2i_bench.log 2>&1 || break
done
