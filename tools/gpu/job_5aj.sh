# masked attention backward: the chunk dQ reduce fused into bwd2's last workgroup (fuse) vs the separate pass
# (nofuse = option mattn_dq_fuse=0, same build), kernel-traced and alternating; then the decoder / long-key tests.
set -o pipefail
cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out && export TMPDIR=/tmp
run() {  # tag opts...
  tag=$1; shift
  cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace -d "$GRAFT_REPO_ROOT/gpurun_out/r5aj_prof_$tag" -o mattn -- python3 "$GRAFT_REPO_ROOT/tools/mattn_bench.py" "$@" > "$GRAFT_REPO_ROOT/gpurun_out/r5aj_mattn_$tag.log" 2>&1
  rc=$?; cd "$GRAFT_REPO_ROOT"; return $rc
}
run nofuse --opt mattn_dq_fuse=0 && run fuse && run nofuse2 --opt mattn_dq_fuse=0 && run fuse2 || exit 1
python3 tools/mattn_levels.py gpurun_out/r5aj_prof_{nofuse,fuse,nofuse2,fuse2}/mattn_results.db > gpurun_out/r5aj_levels.txt || exit 1
rm -rf gpurun_out/r5aj_prof_*
timeout -k 10 600 python -u -m pytest tests/test_decoder_gpu.py tests/test_modules_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r5aj_tests.log 2>&1 || exit 1
timeout -k 10 600 python -u -m pytest tests/test_scale_gpu.py -m gpu -x -q --timeout 300 --timeout-method thread -k "masked_attention or config4 or config5" >> gpurun_out/r5aj_tests.log 2>&1
