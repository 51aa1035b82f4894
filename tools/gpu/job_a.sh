set -o pipefail
cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out && export TMPDIR=/tmp
timeout -k 10 400 python -u tools/step_budget.py --steps 2 --out gpurun_out/a_budget > gpurun_out/a_budget.log 2>&1 || exit 1
timeout -k 10 300 python -u bench.py --no-modes --no-cpu-baseline --no-dropin > gpurun_out/a_bench.json 2> gpurun_out/a_bench.err || exit 1
