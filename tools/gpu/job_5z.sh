# Round-5 final tree, part 1: GPU suite + smoke, the default bench line (CPU baseline, modes, drop-in, peaks)
set -o pipefail
cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out && export TMPDIR=/tmp
bash tools/gpu/tests.sh > gpurun_out/z_tests_tail.log 2>&1 || exit 1
timeout -k 10 600 python -u bench.py > gpurun_out/z_bench.json 2> gpurun_out/z_bench.err
