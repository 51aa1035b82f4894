set -o pipefail
timeout -k 10 300 python -m pytest tests/test_decoder_gpu.py -x -q > gpurun_out/pytest13.log 2>&1 && \
timeout -k 10 300 python tools/step_breakdown.py > gpurun_out/brk13_base.log 2>&1 && \
M2F_CHANNELS_LAST=1 timeout -k 10 300 python tools/step_breakdown.py > gpurun_out/brk13_cl.log 2>&1 && \
timeout -k 10 300 python tools/op_profile.py --rows 60 --attribute > gpurun_out/opprof13.log 2>&1
