set -o pipefail
timeout -k 10 300 python tools/op_profile.py --rows 5 --shapes convolution > gpurun_out/opprof19.log 2>&1 && \
MIOPEN_FIND_MODE=NORMAL timeout -k 10 700 python tools/step_breakdown.py --steps 4 > gpurun_out/brk19_normal.log 2>&1
