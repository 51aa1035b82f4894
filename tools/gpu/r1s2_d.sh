set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
timeout -k 10 400 python -u -m pytest tests -x -q -m gpu --timeout 120 --timeout-method thread > gpurun_out/s2d_tests.log 2>&1; echo "tests rc=$?" >> gpurun_out/s2d_tests.log
timeout -k 10 300 python bench.py --no-cpu-baseline > gpurun_out/s2d_bench.json 2> gpurun_out/s2d_bench.err
timeout -k 10 300 python tools/step_breakdown.py > gpurun_out/s2d_breakdown.log 2>&1
