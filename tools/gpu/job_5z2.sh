# Round-5 final tree, part 2: the new XCD-mapping test, configs 4 / 5, the rocprof kernel trace + stats of the bench,
# FETCH / WRITE / SQ counter passes
set -o pipefail
cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out && export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_scale_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread -k "xcd_mapping" > gpurun_out/z2_tests.log 2>&1 || exit 1
for c in 4 5; do timeout -k 10 300 python -u bench.py --config $c --no-dropin --no-peaks > gpurun_out/z_bench_c$c.json 2> gpurun_out/z_bench_c$c.err || exit 1; done
bash tools/gpu/kernel_stats.sh || exit 1
bash tools/gpu/pmc.sh
