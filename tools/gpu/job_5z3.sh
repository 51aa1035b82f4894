# Round-5 final tree, part 3: the default bench line again (bf16 / fp32 modes on the NCHW backbone) and the step budget
set -o pipefail
cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out && export TMPDIR=/tmp
timeout -k 10 600 python -u bench.py > gpurun_out/z3_bench.json 2> gpurun_out/z3_bench.err || exit 1
timeout -k 10 400 python -u tools/step_budget.py --steps 2 --no-sites --out gpurun_out/z3_budget > gpurun_out/z3_budget.log 2>&1
