# final tree after the 96-wide 8-wave x3 NT default for N = 288: GPU suite + smoke, the default bench line, the step budget
set -o pipefail
cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out && export TMPDIR=/tmp
bash tools/gpu/tests.sh > gpurun_out/ai_tests_tail.log 2>&1 || exit 1
timeout -k 10 600 python -u bench.py > gpurun_out/ai_bench.json 2> gpurun_out/ai_bench.err || exit 1
timeout -k 10 400 python -u tools/step_budget.py --steps 2 --no-sites --out gpurun_out/ai_budget > gpurun_out/ai_budget.log 2>&1
