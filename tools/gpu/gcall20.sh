set -o pipefail
B="timeout -k 10 100 python tools/msda_bench.py --iters 10 --bwd-only"
$B > gpurun_out/abl20_base.log 2>&1 && \
M2F_MSDA_ABLATE=1 $B > gpurun_out/abl20_1.log 2>&1 && \
M2F_MSDA_ABLATE=5 $B > gpurun_out/abl20_5.log 2>&1 && \
M2F_MSDA_ABLATE=7 $B > gpurun_out/abl20_7.log 2>&1 && \
timeout -k 10 300 python tools/op_profile.py --rows 5 --shapes convolution > gpurun_out/opprof19.log 2>&1 && \
MIOPEN_FIND_MODE=NORMAL timeout -k 10 700 python tools/step_breakdown.py --steps 4 > gpurun_out/brk19_normal.log 2>&1
