# Round 2: scale-parity tests (fused MSDA on the 1024^2 pyramid, long-key masked attention, configs 4/5 per rank,
# DDP over RCCL) + module fixtures, then the bench with the new contract fields.
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R && mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests/test_scale_gpu.py tests/test_modules_gpu.py -v --timeout 300 --timeout-method thread > gpurun_out/r2b_tests.log 2>&1
rc=$?
echo "tests rc=$rc"; grep -E "PASSED|FAILED|ERROR" gpurun_out/r2b_tests.log | cut -c1-150
case $rc in 0|1) ;; *) exit $rc;; esac
timeout -k 10 600 python -u bench.py > gpurun_out/r2b_bench.log 2>&1
rc=$?; echo "bench rc=$rc"; tail -c 3000 gpurun_out/r2b_bench.log
