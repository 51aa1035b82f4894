# round 3, call u: MSDA tests and a same-box A/B of the backward (base = r03_t build; new = per-level box
# reduction over that level's lanes), then the full GPU suite + smoke and the default bench line at this build
set -o pipefail
R=$GRAFT_REPO_ROOT
cd "$R" && mkdir -p gpurun_out && export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_msda_gpu.py tests/test_scale_gpu.py -k "fused or nonfinite or msda or tiled or deterministic" \
  -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/tests_u1.log 2>&1 && echo "[u] msda tests ok" && \
for v in base new base new; do
  cp tools/gpu/scratch/libbm2f_$v.so bm2f_amd/lib/libbm2f.so && echo "== $v" >> gpurun_out/mb_u.log && \
  timeout -k 10 120 python -u tools/msda_bench.py --fused --bwd-only >> gpurun_out/mb_u.log 2>&1 || exit 1
done && cp tools/gpu/scratch/libbm2f_new.so bm2f_amd/lib/libbm2f.so && echo "[u] ab ok" && \
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 200 --timeout-method thread > gpurun_out/tests_u.log 2>&1 && \
echo "[u] tests ok" && \
timeout -k 10 200 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke_u.log 2>&1 && echo "[u] smoke ok" && \
timeout -k 10 500 python -u bench.py > gpurun_out/bench_u.json 2> gpurun_out/bench_u.err && echo "[u] bench ok"
