set -o pipefail
R=$GRAFT_REPO_ROOT
cd /tmp && export TMPDIR=/tmp
for a in 0 2; do
B="python3 $R/tools/msda_bench.py --bwd-only --iters 3"
M2F_MSDA_ABLATE=$a timeout -s KILL 90 rocprofv3 --kernel-include-regex msda_bwd --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS --output-format csv -d $R/gpurun_out/pmc_b1_$a -o p -- $B > $R/gpurun_out/pmc_b1_$a.log 2>&1 || exit 1
M2F_MSDA_ABLATE=$a timeout -s KILL 90 rocprofv3 --kernel-include-regex msda_bwd --pmc SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_ACTIVE_INST_VMEM SQ_INSTS_SALU --output-format csv -d $R/gpurun_out/pmc_b2_$a -o p -- $B > $R/gpurun_out/pmc_b2_$a.log 2>&1 || exit 1
M2F_MSDA_ABLATE=$a timeout -s KILL 90 rocprofv3 --kernel-include-regex msda_bwd --pmc SQ_INSTS_VALU_ADD_F64 SQ_INSTS_VALU_CVT SQ_INSTS_VALU_TRANS_F32 SQ_INSTS_VALU_MUL_F32 SQ_WAIT_INST_LDS SQ_INST_CYCLES_VMEM GRBM_GUI_ACTIVE --output-format csv -d $R/gpurun_out/pmc_b3_$a -o p -- $B > $R/gpurun_out/pmc_b3_$a.log 2>&1 || echo "pass3 failed $a"
done
