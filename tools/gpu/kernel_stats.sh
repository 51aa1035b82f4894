# rocprofv3 kernel trace + per-kernel stats of a short bench run (1 warm-up + 3 timed steps, no extra
# instrumented steps) -> gpurun_out/kt/kt_kernel_stats.csv (copy to profiles/rNN_x_kernel_stats.csv).
set -o pipefail
R=$GRAFT_REPO_ROOT
cd "$R" && mkdir -p gpurun_out && export TMPDIR=/tmp
timeout -s KILL 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$R/gpurun_out/kt" -o kt -- \
  python3 "$R/bench.py" --steps 3 --warmup 1 --no-cpu-baseline --no-modes --kernel-steps 0 > gpurun_out/kt.log 2>&1
