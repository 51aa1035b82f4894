# round 3, call v: forward tests (points-per-batch variants) and the fused forward timed at 1 / 2 / 4 points per
# load batch, alternating, plus the op-level forward
set -o pipefail
R=$GRAFT_REPO_ROOT
cd "$R" && mkdir -p gpurun_out && export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_msda_gpu.py -k "forward or fp32 or fixture" -m gpu -x -q --timeout 200 \
  --timeout-method thread > gpurun_out/tests_v.log 2>&1 && echo "[v] tests ok" && \
for pb in 2 1 4 2 1 4; do
  timeout -k 10 120 python -u tools/msda_bench.py --fused --opt msda_fwd_pb=$pb >> gpurun_out/mb_v.log 2>&1 || exit 1
done && echo "[v] bench ok"
