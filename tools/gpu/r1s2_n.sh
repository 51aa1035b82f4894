set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
timeout -k 10 300 python -u -m pytest tests/test_msda_gpu.py -x -q -m gpu --timeout 120 --timeout-method thread > gpurun_out/s2n_tests.log 2>&1; echo "tests rc=$?" >> gpurun_out/s2n_tests.log
timeout -k 10 120 python tools/msda_bench.py --bwd-only > gpurun_out/s2n_bench.log 2>&1
timeout -k 10 300 python bench.py --no-cpu-baseline > gpurun_out/s2n_bench.json 2> gpurun_out/s2n_bench.err
