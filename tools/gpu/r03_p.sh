# round 3, call p: deterministic-mode tests and the MSDA tests, then the backward in default / deterministic mode
set -o pipefail
R=$GRAFT_REPO_ROOT
cd "$R" && mkdir -p gpurun_out && export TMPDIR=/tmp
timeout -k 10 500 python -u -m pytest tests/test_scale_gpu.py tests/test_msda_gpu.py -k "deterministic or fused or repeatable or nonfinite or tiled" \
  -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/tests_p.log 2>&1; rc=$?; tail -3 gpurun_out/tests_p.log
echo "[p] tests rc=$rc"
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
for o in 0 1 0 1; do
  timeout -k 10 120 python -u tools/msda_bench.py --fused --bwd-only --opt msda_bwd_det=$o >> gpurun_out/mb_p.log 2>&1 || exit 1
done
timeout -k 10 120 python -u tools/msda_bench.py --fused --bwd-only --noise 4 --opt msda_bwd_det=1 >> gpurun_out/mb_p.log 2>&1 && echo "[p] bench ok"
