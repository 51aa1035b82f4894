# SQ counters of the fused MSDA kernels (tools/msda_bench.py --fused), two passes:
# issue mix (VALU / LDS / VMEM / SALU instructions, LDS bank conflicts) and where wave time goes.
set -o pipefail
R=$GRAFT_REPO_ROOT
cd "$R" && mkdir -p gpurun_out && export TMPDIR=/tmp
B="python3 $R/tools/msda_bench.py --fused --iters 3"
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_SALU \
  SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE --output-format csv -d "$R/gpurun_out/pmc_m1" -o m1 -- $B > gpurun_out/pmc_m1.log 2>&1 && \
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU \
  SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VMEM GRBM_GUI_ACTIVE --output-format csv -d "$R/gpurun_out/pmc_m2" -o m2 -- $B > gpurun_out/pmc_m2.log 2>&1
