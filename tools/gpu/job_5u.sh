# LDS bank-conflict and issue counters over one bench step (every kernel of the step), for conflict hunting
set -o pipefail
cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out && export TMPDIR=/tmp
PMC_TAG=r5u_step PMC_CMD="python3 $GRAFT_REPO_ROOT/bench.py --steps 1 --warmup 1 --no-cpu-baseline --no-modes --no-dropin --no-peaks --kernel-steps 0" bash tools/gpu/pmc_pass.sh lds issue
