set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R && mkdir -p gpurun_out && export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_msda_gpu.py tests/test_scale_gpu.py -k "msda or tiled or fused or slice or full_size or nonfinite" -q --timeout 120 --timeout-method thread 2>&1 | tee gpurun_out/r2l_tests.log | tail -3
timeout -k 10 600 python -u bench.py --no-cpu-baseline --no-modes > gpurun_out/r2l_bench.log 2>&1; echo "bench rc=$?"
grep -o '"value": [0-9.]*, "unit": "images/s", "n_gpus": 1, "steps": 10, "warmup": 3, "ms_per_step": [0-9.]*' gpurun_out/r2l_bench.log
