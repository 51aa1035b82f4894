set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
timeout -k 10 300 python -u -m pytest tests/test_modules_gpu.py -x -q --timeout 120 --timeout-method thread > gpurun_out/s5v_tests.log 2>&1 || { echo "tests failed"; tail -40 gpurun_out/s5v_tests.log; exit 1; }
tail -1 gpurun_out/s5v_tests.log
timeout -k 10 300 python -u bench.py --no-cpu-baseline > gpurun_out/s5v_bench.log 2>&1 || { tail -30 gpurun_out/s5v_bench.log; exit 1; }
python -c "import json; d=json.loads(open('gpurun_out/s5v_bench.log').read().strip().splitlines()[-1]); print("tn", d['ms_per_step'], d['kernels']['msda_fwd'])"
M2F_CONV3_WGRAD=miopen timeout -k 10 300 python -u bench.py --no-cpu-baseline > gpurun_out/s5v_bench0.log 2>&1 || { tail -30 gpurun_out/s5v_bench0.log; exit 1; }
python -c "import json; d=json.loads(open('gpurun_out/s5v_bench0.log').read().strip().splitlines()[-1]); print("miopen", d['ms_per_step'], d['kernels']['msda_fwd'])"
