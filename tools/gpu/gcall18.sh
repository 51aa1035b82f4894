set -o pipefail
timeout -k 10 300 python tools/gemm_bench.py > gpurun_out/gemm3.log 2>&1 && \
timeout -k 10 300 python -m pytest tests/test_linear_gpu.py -x -q > gpurun_out/pytest18.log 2>&1 && \
timeout -k 10 300 python tools/step_breakdown.py > gpurun_out/brk18.log 2>&1
