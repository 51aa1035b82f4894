# masked attention SQ counters (issue / wait / LDS / MFMA co-issue / MFMA busy) over tools/mattn_bench.py
set -o pipefail
cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out && export TMPDIR=/tmp
PMC_TAG=r5r_mattn PMC_CMD="python3 tools/mattn_bench.py" bash tools/gpu/pmc_pass.sh issue wait lds coexec mfma
