# Round 2: new tiled MSDA backward (sample descriptors, per-cell lists, fp32 walk): parity + timing.
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R && mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_msda_gpu.py tests/test_scale_gpu.py -k "msda or tiled or fused or testpy or slice or fp32_vs or gradcheck or errors or full_size or nonfinite" -v --timeout 120 --timeout-method thread 2>&1 | tee gpurun_out/r2c_tests.log | grep --line-buffered -E "PASSED|FAILED|ERROR"
rc=$?
echo "tests rc=$rc"
case $rc in 0|1) ;; *) exit $rc;; esac
timeout -k 10 120 python -u tools/msda_bench.py --bwd-only > gpurun_out/r2c_mb.log 2>&1; echo "mb rc=$?"; cat gpurun_out/r2c_mb.log | tail -2
timeout -k 10 600 python -u bench.py --no-cpu-baseline --no-modes > gpurun_out/r2c_bench.log 2>&1
rc=$?; echo "bench rc=$rc"; tail -c 1500 gpurun_out/r2c_bench.log
