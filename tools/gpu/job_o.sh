# masked attention backward, two key tiles per wave (mattn_bwd2_kernel) with dQacc over the K / V images (two
# workgroups per CU): correctness (decoder fixtures, ragged / chunked key-tile cases, long keys), then a
# kernel-traced A/B of one key tile vs two in one build
set -o pipefail
cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out && export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_decoder_gpu.py tests/test_modules_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r5o_tests.log 2>&1 || exit 1
timeout -k 10 600 python -u -m pytest tests/test_scale_gpu.py -m gpu -x -q --timeout 300 --timeout-method thread -k "masked_attention or config4 or config5" >> gpurun_out/r5o_tests.log 2>&1 || exit 1
run() {  # tag opts...
  tag=$1; shift
  cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace -d "$GRAFT_REPO_ROOT/gpurun_out/r5o_prof_$tag" -o mattn -- python3 "$GRAFT_REPO_ROOT/tools/mattn_bench.py" "$@" > "$GRAFT_REPO_ROOT/gpurun_out/r5o_mattn_$tag.log" 2>&1
  rc=$?; cd "$GRAFT_REPO_ROOT"; return $rc
}
run keys16 --opt mattn_bwd_keys=16 && run keys32
