# round 3, call i: decoder / module / scale tests with the batched weight cast, then the bench line
set -o pipefail
R=$GRAFT_REPO_ROOT
cd "$R" && mkdir -p gpurun_out && export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_decoder_gpu.py tests/test_modules_gpu.py tests/test_scale_gpu.py \
  tests/test_mask_heads_gpu.py -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/tests_i.log 2>&1 && echo "[i] tests ok" && \
timeout -k 10 400 python -u bench.py --no-cpu-baseline > gpurun_out/bench_i.json 2> gpurun_out/bench_i.err && echo "[i] bench ok" && \
timeout -k 10 300 python -u bench.py --config 4 --steps 10 --warmup 3 --no-peaks > gpurun_out/bench_i4.json 2> gpurun_out/bench_i4.err && \
timeout -k 10 300 python -u bench.py --config 5 --steps 10 --warmup 3 --no-peaks > gpurun_out/bench_i5.json 2> gpurun_out/bench_i5.err && echo "[i] c45 ok"
