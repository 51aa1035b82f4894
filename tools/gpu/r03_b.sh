# round 3, call b: changed-area GPU tests, fp32 find-db entries, fp16/bf16 kernel traces, x3 tile configs, bench
set -o pipefail
R=$GRAFT_REPO_ROOT
cd "$R" && mkdir -p gpurun_out/db && export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_backbone_ops_gpu.py tests/test_mask_heads_gpu.py tests/test_msda_gpu.py \
  -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/tests_b.log 2>&1 && echo "[b] tests ok" && \
cp bm2f_amd/miopen_db/*.ufdb.txt gpurun_out/db/ && \
MIOPEN_FIND_MODE=NORMAL MIOPEN_USER_DB_PATH="$R/gpurun_out/db" timeout -k 10 500 python -u bench.py --amp none \
  --steps 1 --warmup 1 --no-modes --no-cpu-baseline --no-peaks --kernel-steps 0 > gpurun_out/db_fp32.log 2>&1 && \
echo "[b] fp32 search done" && \
timeout -s KILL 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$R/gpurun_out/kt16" -o kt -- \
  python3 "$R/bench.py" --steps 3 --warmup 1 --no-cpu-baseline --no-modes --no-peaks --kernel-steps 0 > gpurun_out/kt16.log 2>&1 && \
timeout -s KILL 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$R/gpurun_out/kt_bf16" -o kt -- \
  python3 "$R/bench.py" --amp bf16 --steps 3 --warmup 1 --no-cpu-baseline --no-modes --no-peaks --kernel-steps 0 > gpurun_out/kt_bf16.log 2>&1 && \
echo "[b] traces done" && \
timeout -k 10 300 python -u tools/gemm_x3_bench.py --x3-only --cfgs 0,2,3 > gpurun_out/mb_x3.log 2>&1 && \
MIOPEN_USER_DB_PATH="$R/gpurun_out/db" timeout -k 10 400 python -u bench.py --no-cpu-baseline \
  > gpurun_out/bench.json 2> gpurun_out/bench.err
