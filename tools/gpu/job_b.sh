set -o pipefail
cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out && export TMPDIR=/tmp
timeout -k 10 400 python -u tools/step_budget.py --steps 2 --out gpurun_out/r5b_budget > gpurun_out/r5b_budget.log 2>&1 || exit 1
