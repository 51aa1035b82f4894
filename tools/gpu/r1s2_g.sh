set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
timeout -k 10 300 python -u -m pytest tests/test_msda_gpu.py tests/test_modules_gpu.py -x -q -m gpu --timeout 120 --timeout-method thread > gpurun_out/s2g_tests.log 2>&1; echo "tests rc=$?" >> gpurun_out/s2g_tests.log
for t in 16 14 12; do M2F_MSDA_TILE=$t timeout -k 10 120 python tools/msda_bench.py --bwd-only >> gpurun_out/s2g_bench.log 2>&1; done
timeout -k 10 300 python bench.py --no-cpu-baseline > gpurun_out/s2g_bench.json 2> gpurun_out/s2g_bench.err
