# round 3, call t: MSDA tests at this build, the default bench line, the config 4 / 5 lines, and the kernel trace +
# FETCH / WRITE passes of one step
set -o pipefail
R=$GRAFT_REPO_ROOT
cd "$R" && mkdir -p gpurun_out && export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_msda_gpu.py tests/test_scale_gpu.py -m gpu -x -q --timeout 200 --timeout-method thread \
  > gpurun_out/tests_t.log 2>&1 && echo "[t] tests ok" && \
for v in base new base new; do
  cp tools/gpu/scratch/libbm2f_$v.so bm2f_amd/lib/libbm2f.so && echo "== $v" >> gpurun_out/mb_t.log && \
  timeout -k 10 120 python -u tools/msda_bench.py --fused --bwd-only >> gpurun_out/mb_t.log 2>&1 || exit 1
done && cp tools/gpu/scratch/libbm2f_new.so bm2f_amd/lib/libbm2f.so && \
timeout -k 10 500 python -u bench.py > gpurun_out/bench_t.json 2> gpurun_out/bench_t.err && echo "[t] bench ok" && \
timeout -k 10 300 python -u bench.py --config 4 --steps 10 --warmup 3 --no-peaks > gpurun_out/bench_t4.json 2> gpurun_out/bench_t4.err && \
timeout -k 10 300 python -u bench.py --config 5 --steps 10 --warmup 3 --no-peaks > gpurun_out/bench_t5.json 2> gpurun_out/bench_t5.err && echo "[t] c45 ok" && \
timeout -s KILL 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$R/gpurun_out/kt_t" -o kt -- \
  python3 "$R/bench.py" --steps 3 --warmup 1 --no-cpu-baseline --no-modes --no-peaks --no-dropin --kernel-steps 0 > gpurun_out/kt_t.log 2>&1 && \
echo "[t] trace ok" && \
B="python3 $R/bench.py --steps 1 --warmup 1 --no-cpu-baseline --no-modes --no-peaks --no-dropin --kernel-steps 0" && \
timeout -s KILL 300 rocprofv3 --pmc FETCH_SIZE GRBM_GUI_ACTIVE --output-format csv -d "$R/gpurun_out/pmc_fetch_t" -o fetch -- $B > gpurun_out/pmc_fetch_t.log 2>&1 && \
timeout -s KILL 300 rocprofv3 --pmc WRITE_SIZE GRBM_GUI_ACTIVE --output-format csv -d "$R/gpurun_out/pmc_write_t" -o write -- $B > gpurun_out/pmc_write_t.log 2>&1 && \
echo "[t] pmc ok"
