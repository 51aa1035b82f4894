# masked attention: one barrier per key block (fwd: double-buffered images already; bwd: two K / V images) --
# correctness, then kernel-traced A/B against the previous build
set -o pipefail
cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out && export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_decoder_gpu.py tests/test_modules_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r5n_tests.log 2>&1 || exit 1
timeout -k 10 600 python -u -m pytest tests/test_scale_gpu.py -m gpu -x -q --timeout 300 --timeout-method thread -k "masked_attention or config4 or config5" >> gpurun_out/r5n_tests.log 2>&1 || exit 1
for lib in tools/lib/libbm2f_mattnbase.so bm2f_amd/lib/libbm2f.so; do
  tag=$(basename $lib .so)
  cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace -d "$GRAFT_REPO_ROOT/gpurun_out/r5n_prof_$tag" -o mattn -- python3 "$GRAFT_REPO_ROOT/tools/mattn_bench.py" --lib "$GRAFT_REPO_ROOT/$lib" > "$GRAFT_REPO_ROOT/gpurun_out/r5n_mattn_$tag.log" 2>&1 || exit 1
  cd "$GRAFT_REPO_ROOT"
done
