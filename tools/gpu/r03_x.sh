# round 3, call x: MSDA tests, then the backward at phase-2 : phase-3 unit ratios 1 / 2 / 3 at the head of the
# merged queue (msda_bwd_ratio), alternating, one library
set -o pipefail
R=$GRAFT_REPO_ROOT
cd "$R" && mkdir -p gpurun_out && export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_msda_gpu.py tests/test_scale_gpu.py -k "fused or nonfinite or msda or tiled or deterministic" \
  -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/tests_x.log 2>&1 && echo "[x] msda tests ok" && \
for r in 1 2 3 1 2 3; do
  timeout -k 10 120 python -u tools/msda_bench.py --fused --bwd-only --opt msda_bwd_ratio=$r >> gpurun_out/mb_x.log 2>&1 || exit 1
done && echo "[x] ab ok"
