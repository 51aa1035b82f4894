# Per-kernel microbenchmarks at the bench shapes: MSDA fwd/bwd, mask heads, x3 GEMMs, x3 convs.
set -o pipefail
cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out && export TMPDIR=/tmp
timeout -k 10 200 python -u tools/msda_bench.py 2>&1 | tee gpurun_out/mb_msda.log && \
timeout -k 10 200 python -u tools/mask_heads_bench.py 2>&1 | tee gpurun_out/mb_mask_heads.log && \
timeout -k 10 300 python -u tools/gemm_x3_bench.py --cfgs "" 2>&1 | tee gpurun_out/mb_gemm_x3.log && \
timeout -k 10 300 python -u tools/conv_bench.py 2>&1 | tee gpurun_out/mb_conv.log
