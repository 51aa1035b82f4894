# masked attention backward: one barrier per key block, two key tiles per wave (mattn_bwd2_kernel) -- correctness
# (decoder fixtures, long-key oracle tests, configs 4 / 5), then kernel-traced A/B: previous build / one key tile /
# two key tiles
set -o pipefail
cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out && export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_decoder_gpu.py tests/test_modules_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r5n_tests.log 2>&1 || exit 1
timeout -k 10 600 python -u -m pytest tests/test_scale_gpu.py -m gpu -x -q --timeout 300 --timeout-method thread -k "masked_attention or config4 or config5" >> gpurun_out/r5n_tests.log 2>&1 || exit 1
run() {  # tag lib opts...
  tag=$1; lib=$2; shift 2
  cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace -d "$GRAFT_REPO_ROOT/gpurun_out/r5n_prof_$tag" -o mattn -- python3 "$GRAFT_REPO_ROOT/tools/mattn_bench.py" --lib "$GRAFT_REPO_ROOT/$lib" "$@" > "$GRAFT_REPO_ROOT/gpurun_out/r5n_mattn_$tag.log" 2>&1
  rc=$?; cd "$GRAFT_REPO_ROOT"; return $rc
}
run base tools/lib/libbm2f_mattnbase.so && run keys16 bm2f_amd/lib/libbm2f.so --opt mattn_bwd_keys=16 && run keys32 bm2f_amd/lib/libbm2f.so
