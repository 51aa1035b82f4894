# round 3, call r: MSDA tests with phases 2/3 in one interleaved work queue, then microbench A/B against the
# previous build (base), the overlap off, and the stamped phase shares (non-overlapped diagnostic build)
set -o pipefail
R=$GRAFT_REPO_ROOT
cd "$R" && mkdir -p gpurun_out && export TMPDIR=/tmp
L=bm2f_amd/lib/libbm2f.so
timeout -k 10 500 python -u -m pytest tests/test_msda_gpu.py tests/test_scale_gpu.py -k "fused or nonfinite or msda or tiled or dropin or fp32 or fixture or gradcheck" \
  -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/tests_r.log 2>&1; rc=$?; tail -3 gpurun_out/tests_r.log
echo "[r] tests rc=$rc"
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
for v in base new base new; do
  cp tools/gpu/scratch/libbm2f_$v.so $L && echo "== $v" >> gpurun_out/mb_r.log && \
  timeout -k 10 120 python -u tools/msda_bench.py --fused --bwd-only >> gpurun_out/mb_r.log 2>&1 && \
  timeout -k 10 120 python -u tools/msda_bench.py --fused --bwd-only --noise 4 >> gpurun_out/mb_r.log 2>&1 || exit 1
done
cp tools/gpu/scratch/libbm2f_new.so $L && echo "== new, overlap off" >> gpurun_out/mb_r.log && \
timeout -k 10 120 python -u tools/msda_bench.py --fused --bwd-only --opt msda_bwd_overlap=0 >> gpurun_out/mb_r.log 2>&1 && \
timeout -k 10 120 python -u tools/msda_bench.py --bwd-only >> gpurun_out/mb_r.log 2>&1 && echo "[r] bench ok"
