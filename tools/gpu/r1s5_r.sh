set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
timeout -k 10 300 python -u -m pytest tests/test_msda_gpu.py tests/test_modules_gpu.py -x -q --timeout 120 --timeout-method thread > gpurun_out/s5r_tests.log 2>&1 || { echo "tests failed"; tail -40 gpurun_out/s5r_tests.log; exit 1; }
tail -1 gpurun_out/s5r_tests.log
timeout -k 10 300 python -u bench.py --no-cpu-baseline > gpurun_out/s5r_bench.log 2>&1 || { tail -30 gpurun_out/s5r_bench.log; exit 1; }
python -c "import json; d=json.loads(open('gpurun_out/s5r_bench.log').read().strip().splitlines()[-1]); print('headmajor', d['ms_per_step'], d['kernels']['msda_bwd'])"
M2F_MSDA_BWD_HEAD_MAJOR=0 timeout -k 10 300 python -u bench.py --no-cpu-baseline > gpurun_out/s5r_bench0.log 2>&1 || { tail -30 gpurun_out/s5r_bench0.log; exit 1; }
python -c "import json; d=json.loads(open('gpurun_out/s5r_bench0.log').read().strip().splitlines()[-1]); print('unheadmajor', d['ms_per_step'], d['kernels']['msda_bwd'])"
