set -o pipefail
timeout -k 10 300 python -m pytest tests/test_linear_gpu.py tests/test_norm_gpu.py tests/test_modules_gpu.py tests/test_msda_gpu.py -x -q > gpurun_out/pytest16.log 2>&1 && \
timeout -k 10 300 python tools/step_breakdown.py > gpurun_out/brk16.log 2>&1 && \
timeout -k 10 300 python tools/op_profile.py --rows 40 --attribute > gpurun_out/opprof16.log 2>&1
