# round 3, call d: masked-attention dQ paths A/B, channels-last backbone A/B, tests of the changed kernels
set -o pipefail
R=$GRAFT_REPO_ROOT
cd "$R" && mkdir -p gpurun_out && export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_scale_gpu.py -k "masked_attention" tests/test_decoder_gpu.py tests/test_modules_gpu.py \
  tests/test_mask_heads_gpu.py -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/tests_d.log 2>&1 && echo "[d] tests ok" && \
timeout -k 10 200 python -u tools/mattn_bench.py > gpurun_out/mattn_new.log 2>&1 && \
timeout -k 10 200 python -u tools/mattn_bench.py --dq-atomic > gpurun_out/mattn_atomic.log 2>&1 && echo "[d] mattn ok" && \
timeout -k 10 300 python -u bench.py --no-cpu-baseline --no-modes --no-peaks --no-dropin --channels-last 1 > gpurun_out/bench_cl.json 2> gpurun_out/bench_cl.err && \
timeout -k 10 300 python -u bench.py --no-cpu-baseline --no-modes --no-peaks --no-dropin --channels-last 0 > gpurun_out/bench_ncl.json 2> gpurun_out/bench_ncl.err && \
timeout -k 10 300 python -u bench.py --config 4 --steps 10 --warmup 3 > gpurun_out/bench_d4.json 2> gpurun_out/bench_d4.err && echo "[d] bench ok"
