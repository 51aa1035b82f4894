# round 3, call k: MSDA tests with the quad-form kernels (fwd, bwd phase 2, new phase 3), then microbench A/B:
# HEAD library (base) vs this build (new; and new with the quad forms off), reference-init and noise-4 sampling,
# then the stamped phase shares of the new backward
set -o pipefail
R=$GRAFT_REPO_ROOT
cd "$R" && mkdir -p gpurun_out && export TMPDIR=/tmp
L=bm2f_amd/lib/libbm2f.so
timeout -k 10 500 python -u -m pytest tests/test_msda_gpu.py tests/test_scale_gpu.py -k "fused or nonfinite or msda or tiled or dropin or fp32 or fixture or gradcheck" \
  -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/tests_k.log 2>&1; rc=$?; tail -3 gpurun_out/tests_k.log
echo "[k] tests rc=$rc"
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
for v in base new base new; do
  cp tools/gpu/scratch/libbm2f_$v.so $L && echo "== $v" >> gpurun_out/mb_k.log && \
  timeout -k 10 120 python -u tools/msda_bench.py --fused >> gpurun_out/mb_k.log 2>&1 && \
  timeout -k 10 120 python -u tools/msda_bench.py --fused --noise 4 >> gpurun_out/mb_k.log 2>&1 && \
  timeout -k 10 120 python -u tools/msda_bench.py >> gpurun_out/mb_k.log 2>&1 || exit 1
done
cp tools/gpu/scratch/libbm2f_new.so $L && echo "== new, quad off" >> gpurun_out/mb_k.log && \
timeout -k 10 120 python -u tools/msda_bench.py --fused --opt msda_fwd_quad=0 --opt msda_bwd_quad=0 >> gpurun_out/mb_k.log 2>&1 && \
timeout -k 10 120 python -u tools/msda_stamps.py > gpurun_out/stamps_k.log 2>&1 && echo "[k] bench ok"
