# masked attention forward combine: a thread per (row, 4 channels) (c0 = option mattn_combine=0) vs a wave per row
# (c1 = forced everywhere; dflt = the default, the wave form from 16 chunks), kernel-traced and alternating; then tests.
set -o pipefail
cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out && export TMPDIR=/tmp
run() {  # tag opts...
  tag=$1; shift
  cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace -d "$GRAFT_REPO_ROOT/gpurun_out/r5ak_prof_$tag" -o mattn -- python3 "$GRAFT_REPO_ROOT/tools/mattn_bench.py" "$@" > "$GRAFT_REPO_ROOT/gpurun_out/r5ak_mattn_$tag.log" 2>&1
  rc=$?; cd "$GRAFT_REPO_ROOT"; return $rc
}
timeout -k 10 600 python -u -m pytest tests/test_scale_gpu.py -m gpu -x -q --timeout 300 --timeout-method thread -k "combine" > gpurun_out/r5ak_tests.log 2>&1 || exit 1
run c0 --opt mattn_combine=0 && run c1 --opt mattn_combine=1 && run dflt && run c0b --opt mattn_combine=0 && run c1b --opt mattn_combine=1 && run dfltb || exit 1
python3 tools/mattn_levels.py gpurun_out/r5ak_prof_{c0,c1,dflt,c0b,c1b,dfltb}/mattn_results.db > gpurun_out/r5ak_levels.txt || exit 1
rm -rf gpurun_out/r5ak_prof_*
timeout -k 10 600 python -u -m pytest tests/test_decoder_gpu.py tests/test_modules_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread >> gpurun_out/r5ak_tests.log 2>&1 || exit 1
timeout -k 10 600 python -u -m pytest tests/test_scale_gpu.py -m gpu -x -q --timeout 300 --timeout-method thread -k "masked_attention or config4 or config5" >> gpurun_out/r5ak_tests.log 2>&1
