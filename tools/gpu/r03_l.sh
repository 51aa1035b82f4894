# round 3, call l: SQ counter passes over the quad-form fused MSDA kernels (issue mix, LDS, waits), one rocprofv3
# run per pass, then a third pass on the fused kernels with the quad forms off for comparison
set -o pipefail
R=$GRAFT_REPO_ROOT
cd "$R" && mkdir -p gpurun_out && export TMPDIR=/tmp
B="python3 $R/tools/msda_bench.py --fused --iters 3"
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_SALU \
  SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE --output-format csv -d "$R/gpurun_out/pmc_l1" -o m1 -- $B > gpurun_out/pmc_l1.log 2>&1 && \
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU \
  SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VMEM GRBM_GUI_ACTIVE --output-format csv -d "$R/gpurun_out/pmc_l2" -o m2 -- $B > gpurun_out/pmc_l2.log 2>&1 && \
timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU \
  GRBM_GUI_ACTIVE --output-format csv -d "$R/gpurun_out/pmc_l3" -o m3 -- $B --opt msda_fwd_quad=0 --opt msda_bwd_quad=0 > gpurun_out/pmc_l3.log 2>&1 && \
echo "[l] pmc ok"
