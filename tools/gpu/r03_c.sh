# round 3, call c: changed tests (scale incl. drop-in / config-4 oracle / crossing checks, msda, linear bits),
# then the bench line (config 2 with drop-in timing and peaks) and the config 4 / 5 per-rank lines
set -o pipefail
R=$GRAFT_REPO_ROOT
cd "$R" && mkdir -p gpurun_out && export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests/test_scale_gpu.py tests/test_msda_gpu.py tests/test_linear_gpu.py tests/test_mask_heads_gpu.py \
  tests/test_backbone_ops_gpu.py -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/tests_c.log 2>&1 && \
echo "[c] tests ok" && \
timeout -k 10 400 python -u bench.py --no-cpu-baseline > gpurun_out/bench_c2.json 2> gpurun_out/bench_c2.err && \
echo "[c] config 2 ok" && \
timeout -k 10 300 python -u bench.py --config 4 --steps 10 --warmup 3 > gpurun_out/bench_c4.json 2> gpurun_out/bench_c4.err && \
echo "[c] config 4 ok" && \
timeout -k 10 300 python -u bench.py --config 5 --steps 10 --warmup 3 > gpurun_out/bench_c5.json 2> gpurun_out/bench_c5.err && \
echo "[c] config 5 ok"
