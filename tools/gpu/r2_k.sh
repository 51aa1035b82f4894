set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R && mkdir -p gpurun_out && export TMPDIR=/tmp
timeout -k 10 120 python -u tools/dbg_msda.py 2>&1 | tee gpurun_out/r2k_dbg.log
for thr in 512 1024; do
M2F_MSDA_THREADS=$thr timeout -k 10 120 python -u tools/msda_stamps.py 2>&1 | tee gpurun_out/r2k_stamps_$thr.log
M2F_MSDA_THREADS=$thr timeout -k 10 120 python -u tools/msda_bench.py --bwd-only 2>&1 | tee gpurun_out/r2k_mb_$thr.log
done
M2F_MSDA_THREADS=512 M2F_MSDA_TILE=8 M2F_MSDA_TILE_W=16 timeout -k 10 120 python -u tools/msda_bench.py --bwd-only 2>&1 | tee gpurun_out/r2k_mb_8x16.log
M2F_MSDA_THREADS=512 M2F_MSDA_TILE=12 M2F_MSDA_TILE_W=12 timeout -k 10 120 python -u tools/msda_bench.py --bwd-only 2>&1 | tee gpurun_out/r2k_mb_12.log
timeout -k 10 600 python -u -m pytest tests/test_msda_gpu.py tests/test_scale_gpu.py -k "msda or tiled or fused or slice or full_size or nonfinite" -q --timeout 120 --timeout-method thread 2>&1 | tee gpurun_out/r2k_tests.log | tail -5
