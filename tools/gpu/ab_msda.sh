# Same-box A/B of the MSDA kernels: tools/gpu/scratch/libbm2f_{base,new}.so (built beforehand in-tree).
# The new library's MSDA GPU tests first, then the microbenchmark alternating base / new.
set -o pipefail
cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out && export TMPDIR=/tmp
L=bm2f_amd/lib/libbm2f.so
cp tools/gpu/scratch/libbm2f_new.so $L && \
{ [ -n "$AB_SKIP_TESTS" ] || timeout -k 10 500 python -u -m pytest tests/test_msda_gpu.py tests/test_scale_gpu.py -x -q --timeout 120 --timeout-method thread ${AB_TESTS_K:+-k "$AB_TESTS_K"} > gpurun_out/ab_tests.log 2>&1; } && \
for v in base new base new; do
  cp tools/gpu/scratch/libbm2f_$v.so $L && echo "== $v" >> gpurun_out/ab_msda.log && \
  timeout -k 10 120 python -u tools/msda_bench.py $AB_BENCH_ARGS >> gpurun_out/ab_msda.log 2>&1 && \
  timeout -k 10 120 python -u tools/msda_bench.py --fused $AB_BENCH_ARGS >> gpurun_out/ab_msda.log 2>&1 || exit 1
done
cp tools/gpu/scratch/libbm2f_new.so $L
