# final tree after the masked-attention forward's lazy rescaling: GPU suite + smoke, the default bench line
set -o pipefail
cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out && export TMPDIR=/tmp
bash tools/gpu/tests.sh > gpurun_out/y_tests_tail.log 2>&1 || exit 1
timeout -k 10 600 python -u bench.py > gpurun_out/y_bench.json 2> gpurun_out/y_bench.err
