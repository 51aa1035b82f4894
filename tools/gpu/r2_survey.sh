# Round-2 counter survey of the round-1 step: list gfx950 counters, then one SQ/GRBM pass over every kernel
# of a short bench run (MFMA busy, VALU/MFMA/LDS instruction counts, wave cycles) for SURVEY §8 row d2.
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R && mkdir -p gpurun_out && export TMPDIR=/tmp
timeout -s KILL 120 rocprofv3 -L > gpurun_out/r2a_counters.txt 2>&1 || echo "list rc=$?"
timeout -s KILL 300 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_WAIT_INST_ANY GRBM_GUI_ACTIVE --output-format csv -d $R/gpurun_out/r2a_sq -o sq -- python3 $R/bench.py --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/r2a_sq.log 2>&1
echo "sq rc=$?"
ls -R gpurun_out/r2a_sq | head
