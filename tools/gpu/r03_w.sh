# round 3, call w: MSDA tests and a same-box A/B of the backward (base = r03_v build; new = phase-2 units spread
# evenly over the merged phase-2/3 queue), default and noise-4 sampling
set -o pipefail
R=$GRAFT_REPO_ROOT
cd "$R" && mkdir -p gpurun_out && export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_msda_gpu.py tests/test_scale_gpu.py -k "fused or nonfinite or msda or tiled or deterministic" \
  -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/tests_w.log 2>&1 && echo "[w] msda tests ok" && \
for v in base new base new base new; do
  cp tools/gpu/scratch/libbm2f_$v.so bm2f_amd/lib/libbm2f.so && echo "== $v" >> gpurun_out/mb_w.log && \
  timeout -k 10 120 python -u tools/msda_bench.py --fused --bwd-only >> gpurun_out/mb_w.log 2>&1 || exit 1
done && \
for v in base new; do
  cp tools/gpu/scratch/libbm2f_$v.so bm2f_amd/lib/libbm2f.so && echo "== $v noise 4" >> gpurun_out/mb_w.log && \
  timeout -k 10 120 python -u tools/msda_bench.py --fused --bwd-only --noise 4 >> gpurun_out/mb_w.log 2>&1 || exit 1
done && cp tools/gpu/scratch/libbm2f_new.so bm2f_amd/lib/libbm2f.so && echo "[w] ab ok"
