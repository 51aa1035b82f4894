# job_5ak's combine A/B again with the level tool counting both combine kernels (tests passed in job_5ak)
set -o pipefail
cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out && export TMPDIR=/tmp
run() {  # tag opts...
  tag=$1; shift
  cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace -d "$GRAFT_REPO_ROOT/gpurun_out/r5al_prof_$tag" -o mattn -- python3 "$GRAFT_REPO_ROOT/tools/mattn_bench.py" "$@" > "$GRAFT_REPO_ROOT/gpurun_out/r5al_mattn_$tag.log" 2>&1
  rc=$?; cd "$GRAFT_REPO_ROOT"; return $rc
}
run c0 --opt mattn_combine=0 && run c1 --opt mattn_combine=1 && run c0b --opt mattn_combine=0 && run c1b --opt mattn_combine=1 || exit 1
python3 tools/mattn_levels.py gpurun_out/r5al_prof_{c0,c1,c0b,c1b}/mattn_results.db > gpurun_out/r5al_levels.txt || exit 1
rm -rf gpurun_out/r5al_prof_*
