set -o pipefail
timeout -k 10 300 python -m pytest tests/test_mask_fold.py tests/test_modules_gpu.py tests/test_decoder_gpu.py -x -q > gpurun_out/pytest14.log 2>&1 && \
timeout -k 10 300 python tools/step_breakdown.py > gpurun_out/brk14.log 2>&1 && \
MIOPEN_FIND_MODE=NORMAL timeout -k 10 600 python tools/step_breakdown.py --steps 5 > gpurun_out/brk14_normal.log 2>&1
