# round 3, call q: kernel trace + per-kernel stats of the bench step (fp16 default), then the FETCH / WRITE / SQ
# counter passes over one step (each its own rocprofv3 run)
set -o pipefail
R=$GRAFT_REPO_ROOT
cd "$R" && mkdir -p gpurun_out && export TMPDIR=/tmp
timeout -s KILL 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$R/gpurun_out/kt_q" -o kt -- \
  python3 "$R/bench.py" --steps 3 --warmup 1 --no-cpu-baseline --no-modes --no-peaks --no-dropin --kernel-steps 0 > gpurun_out/kt_q.log 2>&1 && \
echo "[q] trace ok" && \
B="python3 $R/bench.py --steps 1 --warmup 1 --no-cpu-baseline --no-modes --no-peaks --no-dropin --kernel-steps 0" && \
timeout -s KILL 300 rocprofv3 --pmc FETCH_SIZE GRBM_GUI_ACTIVE --output-format csv -d "$R/gpurun_out/pmc_fetch_q" -o fetch -- $B > gpurun_out/pmc_fetch_q.log 2>&1 && \
timeout -s KILL 300 rocprofv3 --pmc WRITE_SIZE GRBM_GUI_ACTIVE --output-format csv -d "$R/gpurun_out/pmc_write_q" -o write -- $B > gpurun_out/pmc_write_q.log 2>&1 && \
timeout -s KILL 300 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VALU_MFMA_MOPS_BF16 \
  SQ_INSTS_VALU_MFMA_MOPS_F16 SQ_INSTS_VALU_MFMA_MOPS_F32 SQ_WAIT_ANY GRBM_GUI_ACTIVE --output-format csv \
  -d "$R/gpurun_out/pmc_sq_q" -o sq -- $B > gpurun_out/pmc_sq_q.log 2>&1 && echo "[q] pmc ok"
