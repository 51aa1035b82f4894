# masked attention A/B, kernel-traced, alternating: base = previous commit; pk = lazy forward rescaling + explicit
# packed-f32 P / dS math; slp = lazy + scalar code (the in-tree build, compiler SLP on); noslp = the same built with
# -fno-slp-vectorize.  Then the decoder / long-key tests on the in-tree build.
set -o pipefail
cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out && export TMPDIR=/tmp
run() {  # tag opts...
  tag=$1; shift
  cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace -d "$GRAFT_REPO_ROOT/gpurun_out/r5w_prof_$tag" -o mattn -- python3 "$GRAFT_REPO_ROOT/tools/mattn_bench.py" "$@" > "$GRAFT_REPO_ROOT/gpurun_out/r5w_mattn_$tag.log" 2>&1
  rc=$?; cd "$GRAFT_REPO_ROOT"; return $rc
}
L="$GRAFT_REPO_ROOT/tools/lib"
run base --lib "$L/libbm2f_base.so" && run pk --lib "$L/libbm2f_pk.so" && run slp && run noslp --lib "$L/libbm2f_noslp.so" && \
run base2 --lib "$L/libbm2f_base.so" && run pk2 --lib "$L/libbm2f_pk.so" && run slp2 && run noslp2 --lib "$L/libbm2f_noslp.so" || exit 1
# per-level medians here, then drop the trace databases (gpurun copies back at most 64 MiB)
python3 tools/mattn_levels.py gpurun_out/r5w_prof_{base,pk,slp,noslp,base2,pk2,slp2,noslp2}/mattn_results.db > gpurun_out/r5w_levels.txt || exit 1
rm -rf gpurun_out/r5w_prof_*
timeout -k 10 600 python -u -m pytest tests/test_decoder_gpu.py tests/test_modules_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r5w_tests.log 2>&1 || exit 1
timeout -k 10 600 python -u -m pytest tests/test_scale_gpu.py -m gpu -x -q --timeout 300 --timeout-method thread -k "masked_attention or config4 or config5" >> gpurun_out/r5w_tests.log 2>&1
