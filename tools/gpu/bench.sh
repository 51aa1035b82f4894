# The bench line of the round (bench.py defaults: 10 timed steps, roofline_all, AMP fp16 / fp32 modes,
# the CPU baseline) -> gpurun_out/bench.json.   gpurun --timeout 900 -- 'bash tools/gpu/bench.sh'
set -o pipefail
cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out && export TMPDIR=/tmp
timeout -k 10 800 python -u bench.py 2> gpurun_out/bench.err | tee gpurun_out/bench.json
