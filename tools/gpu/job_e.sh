# x3 engine SQ issue / wait / MFMA-coexec counters: the 3x3 conv and the encoder GEMM shapes
set -o pipefail
cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out && export TMPDIR=/tmp
PMC_TAG=x3conv PMC_CMD="python3 tools/conv_bench.py --only layer_1 --x3-only" bash tools/gpu/pmc_pass.sh issue wait coexec lds || exit 1
PMC_TAG=x3gemm PMC_CMD="python3 tools/gemm_x3_bench.py --x3-only --cfgs 3" bash tools/gpu/pmc_pass.sh issue wait coexec lds || exit 1
