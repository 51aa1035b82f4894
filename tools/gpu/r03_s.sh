# round 3, call s: MSDA tests, same-box A/B of the backward (base = the r03_p build; new = LDS g-row swizzle +
# one fewer barrier), then the full GPU suite + smoke, the default bench line, the config 4 / 5 lines, and the
# kernel trace + FETCH / WRITE passes of one step
set -o pipefail
R=$GRAFT_REPO_ROOT
cd "$R" && mkdir -p gpurun_out && export TMPDIR=/tmp
L=bm2f_amd/lib/libbm2f.so
timeout -k 10 400 python -u -m pytest tests/test_msda_gpu.py tests/test_scale_gpu.py -k "fused or nonfinite or msda or tiled or deterministic" \
  -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/tests_s1.log 2>&1; rc=$?; tail -2 gpurun_out/tests_s1.log
echo "[s] msda tests rc=$rc"
[ $rc -eq 0 ] || exit 1
for v in base new base new; do
  cp tools/gpu/scratch/libbm2f_$v.so $L && echo "== $v" >> gpurun_out/mb_s.log && \
  timeout -k 10 120 python -u tools/msda_bench.py --fused --bwd-only >> gpurun_out/mb_s.log 2>&1 || exit 1
done
cp tools/gpu/scratch/libbm2f_new.so $L && echo "[s] ab ok" && \
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 200 --timeout-method thread > gpurun_out/tests_s.log 2>&1 && \
echo "[s] tests ok" && \
timeout -k 10 200 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke_s.log 2>&1 && echo "[s] smoke ok" && \
timeout -k 10 500 python -u bench.py > gpurun_out/bench_s.json 2> gpurun_out/bench_s.err && echo "[s] bench ok" && \
timeout -k 10 300 python -u bench.py --config 4 --steps 10 --warmup 3 --no-peaks > gpurun_out/bench_s4.json 2> gpurun_out/bench_s4.err && \
timeout -k 10 300 python -u bench.py --config 5 --steps 10 --warmup 3 --no-peaks > gpurun_out/bench_s5.json 2> gpurun_out/bench_s5.err && echo "[s] c45 ok" && \
timeout -s KILL 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$R/gpurun_out/kt_s" -o kt -- \
  python3 "$R/bench.py" --steps 3 --warmup 1 --no-cpu-baseline --no-modes --no-peaks --no-dropin --kernel-steps 0 > gpurun_out/kt_s.log 2>&1 && \
echo "[s] trace ok" && \
B="python3 $R/bench.py --steps 1 --warmup 1 --no-cpu-baseline --no-modes --no-peaks --no-dropin --kernel-steps 0" && \
timeout -s KILL 300 rocprofv3 --pmc FETCH_SIZE GRBM_GUI_ACTIVE --output-format csv -d "$R/gpurun_out/pmc_fetch_s" -o fetch -- $B > gpurun_out/pmc_fetch_s.log 2>&1 && \
timeout -s KILL 300 rocprofv3 --pmc WRITE_SIZE GRBM_GUI_ACTIVE --output-format csv -d "$R/gpurun_out/pmc_write_s" -o write -- $B > gpurun_out/pmc_write_s.log 2>&1 && \
echo "[s] pmc ok"
