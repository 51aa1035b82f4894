set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R && mkdir -p gpurun_out && export TMPDIR=/tmp
timeout -k 10 120 python -u tools/dbg_msda.py 2>&1 | tee gpurun_out/r2j_dbg.log
timeout -k 10 120 python -u tools/msda_stamps.py 2>&1 | tee gpurun_out/r2j_stamps.log
timeout -k 10 120 python -u tools/msda_bench.py --bwd-only 2>&1 | tee gpurun_out/r2j_mb.log
timeout -k 10 600 python -u -m pytest tests/test_msda_gpu.py tests/test_scale_gpu.py -k "msda or tiled or fused or slice or full_size or nonfinite" -q --timeout 120 --timeout-method thread 2>&1 | tee gpurun_out/r2j_tests.log | tail -5
