# Counter passes over one bench step, each in its own rocprofv3 run (the per-block counter limits of
# MI355X_MICROARCH.md): HBM fetch, HBM write, and SQ (MFMA busy / MOPS, waves, waits).  Summarise with
#   python tools/pmc_summary.py gpurun_out/pmc_sq/sq_counter_collection.csv gpurun_out/pmc_fetch/fetch_counter_collection.csv \
#          gpurun_out/pmc_write/write_counter_collection.csv --json profiles/rNN_x_pmc_summary.json
set -o pipefail
R=$GRAFT_REPO_ROOT
cd "$R" && mkdir -p gpurun_out && export TMPDIR=/tmp
B="python3 $R/bench.py --steps 1 --warmup 1 --no-cpu-baseline --no-modes --no-dropin --no-peaks --kernel-steps 0"
timeout -s KILL 300 rocprofv3 --pmc FETCH_SIZE GRBM_GUI_ACTIVE --output-format csv -d "$R/gpurun_out/pmc_fetch" -o fetch -- $B > gpurun_out/pmc_fetch.log 2>&1 && \
timeout -s KILL 300 rocprofv3 --pmc WRITE_SIZE GRBM_GUI_ACTIVE --output-format csv -d "$R/gpurun_out/pmc_write" -o write -- $B > gpurun_out/pmc_write.log 2>&1 && \
timeout -s KILL 300 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VALU_MFMA_MOPS_BF16 \
  SQ_INSTS_VALU_MFMA_MOPS_F16 SQ_INSTS_VALU_MFMA_MOPS_F32 SQ_WAIT_ANY GRBM_GUI_ACTIVE --output-format csv \
  -d "$R/gpurun_out/pmc_sq" -o sq -- $B > gpurun_out/pmc_sq.log 2>&1
