# x3 A/B: prefetch loads fenced ahead of the chunk MFMAs (-DM2F_X3_SB) vs the default build, alternating rounds
set -o pipefail
cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out && export TMPDIR=/tmp
for r in 1 2; do
  for lib in bm2f_amd/lib/libbm2f.so tools/lib/libbm2f_x3sb_gemm.so; do
    echo "== round $r gemm $lib" >> gpurun_out/r5h_ab.log
    timeout -k 10 200 python -u tools/gemm_x3_bench.py --x3-only --cfgs "" --lib $lib >> gpurun_out/r5h_ab.log 2>&1 || exit 1
  done
  for lib in bm2f_amd/lib/libbm2f.so tools/lib/libbm2f_x3sb_conv.so; do
    echo "== round $r conv $lib" >> gpurun_out/r5h_ab.log
    timeout -k 10 200 python -u tools/conv_bench.py --x3-only --lib $lib >> gpurun_out/r5h_ab.log 2>&1 || exit 1
  done
done
# masked attention: per-kernel durations (main kernel vs combine / dq reduce) at the decoder shapes
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$GRAFT_REPO_ROOT/gpurun_out/r5h_mattn_prof" -o mattn -- python3 "$GRAFT_REPO_ROOT/tools/mattn_bench.py" > "$GRAFT_REPO_ROOT/gpurun_out/r5h_mattn.log" 2>&1 || exit 1
