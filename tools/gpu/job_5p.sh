# masked attention: the heads of one (image, key chunk) on one XCD (option mattn_xcd) -- correctness (decoder
# fixtures, key-tile / long-key cases), kernel-traced A/B of mattn_xcd 0 / 1, FETCH_SIZE / WRITE_SIZE passes of both
set -o pipefail
cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out && export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_decoder_gpu.py tests/test_modules_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r5p_tests.log 2>&1 || exit 1
timeout -k 10 600 python -u -m pytest tests/test_scale_gpu.py -m gpu -x -q --timeout 300 --timeout-method thread -k "masked_attention or config4 or config5" >> gpurun_out/r5p_tests.log 2>&1 || exit 1
run() {  # tag opts...
  tag=$1; shift
  cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace -d "$GRAFT_REPO_ROOT/gpurun_out/r5p_prof_$tag" -o mattn -- python3 "$GRAFT_REPO_ROOT/tools/mattn_bench.py" "$@" > "$GRAFT_REPO_ROOT/gpurun_out/r5p_mattn_$tag.log" 2>&1
  rc=$?; cd "$GRAFT_REPO_ROOT"; return $rc
}
run xcd0 --opt mattn_xcd=0 && run xcd1 && run xcd1k16 --opt mattn_bwd_keys=16 || exit 1
PMC_TAG=r5p_xcd0 PMC_CMD="python3 tools/mattn_bench.py --opt mattn_xcd=0" bash tools/gpu/pmc_pass.sh fetch write || exit 1
PMC_TAG=r5p_xcd1 PMC_CMD="python3 tools/mattn_bench.py" bash tools/gpu/pmc_pass.sh fetch write
