# Round-5 final tree, part 2: configs 4 / 5, the rocprof kernel trace + stats of the bench, FETCH / WRITE / SQ counter
# passes, the step budget
set -o pipefail
cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out && export TMPDIR=/tmp
for c in 4 5; do timeout -k 10 300 python -u bench.py --config $c --no-dropin --no-peaks > gpurun_out/z_bench_c$c.json 2> gpurun_out/z_bench_c$c.err || exit 1; done
bash tools/gpu/kernel_stats.sh || exit 1
bash tools/gpu/pmc.sh || exit 1
timeout -k 10 400 python -u tools/step_budget.py --steps 2 --no-sites --out gpurun_out/z_budget > gpurun_out/z_budget.log 2>&1
