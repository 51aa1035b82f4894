set -o pipefail
timeout -k 10 400 python -m pytest tests -m gpu -x -q > gpurun_out/pytest12.log 2>&1 && \
timeout -k 10 400 python bench.py > gpurun_out/bench12.json 2> gpurun_out/bench12.err && \
cd /tmp && export TMPDIR=/tmp && \
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/prof12 -o run -- python3 $GRAFT_REPO_ROOT/bench.py --steps 3 --warmup 2 --no-cpu-baseline > $GRAFT_REPO_ROOT/gpurun_out/prof12.log 2>&1
