# masked-attention forward: chunk plans with fewer, longer chunks (no combine pass when one chunk covers the keys);
# kernel durations from the rocprof kernel trace (the bench tool's loop is host-bound at the short levels)
set -o pipefail
cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out && export TMPDIR=/tmp
for mb in 2 4 8 16; do
  cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace -d "$GRAFT_REPO_ROOT/gpurun_out/r5l_prof_$mb" -o mattn -- python3 "$GRAFT_REPO_ROOT/tools/mattn_bench.py" --opt mattn_fwd_minblk=$mb > "$GRAFT_REPO_ROOT/gpurun_out/r5l_mattn_$mb.log" 2>&1 || exit 1
done
