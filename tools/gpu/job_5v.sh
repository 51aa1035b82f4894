# masked-attention forward: lazy rescaling of the online softmax (the running max moves only past 2^8): correctness
# (decoder fixtures, key-tile / long-key cases, configs 4 / 5), kernel-traced A/B against the previous build
set -o pipefail
cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out && export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_decoder_gpu.py tests/test_modules_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r5v_tests.log 2>&1 || exit 1
timeout -k 10 600 python -u -m pytest tests/test_scale_gpu.py -m gpu -x -q --timeout 300 --timeout-method thread -k "masked_attention or config4 or config5" >> gpurun_out/r5v_tests.log 2>&1 || exit 1
run() {  # tag opts...
  tag=$1; shift
  cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace -d "$GRAFT_REPO_ROOT/gpurun_out/r5v_prof_$tag" -o mattn -- python3 "$GRAFT_REPO_ROOT/tools/mattn_bench.py" "$@" > "$GRAFT_REPO_ROOT/gpurun_out/r5v_mattn_$tag.log" 2>&1
  rc=$?; cd "$GRAFT_REPO_ROOT"; return $rc
}
run base --lib "$GRAFT_REPO_ROOT/tools/lib/libbm2f_base.so" && run new && run base2 --lib "$GRAFT_REPO_ROOT/tools/lib/libbm2f_base.so" && run new2
