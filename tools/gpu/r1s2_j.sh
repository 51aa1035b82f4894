set -o pipefail
R=$GRAFT_REPO_ROOT
cd /tmp && export TMPDIR=/tmp
B="python3 $R/tools/msda_bench.py --bwd-only --iters 3"
timeout -s KILL 90 rocprofv3 --kernel-include-regex msda_bwd --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS --output-format csv -d $R/gpurun_out/pmc_j1 -o p -- $B > $R/gpurun_out/pmc_j1.log 2>&1
timeout -s KILL 90 rocprofv3 --kernel-include-regex msda_bwd --pmc SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_ACTIVE_INST_VMEM SQ_INSTS_SALU --output-format csv -d $R/gpurun_out/pmc_j2 -o p -- $B > $R/gpurun_out/pmc_j2.log 2>&1
timeout -s KILL 90 rocprofv3 --kernel-include-regex msda_bwd --pmc FETCH_SIZE GRBM_GUI_ACTIVE --output-format csv -d $R/gpurun_out/pmc_j3 -o p -- $B > $R/gpurun_out/pmc_j3.log 2>&1
timeout -s KILL 90 rocprofv3 --kernel-include-regex msda_bwd --pmc TCC_HIT_sum TCC_MISS_sum --output-format csv -d $R/gpurun_out/pmc_j4 -o p -- $B > $R/gpurun_out/pmc_j4.log 2>&1
ls -R $R/gpurun_out/pmc_j1 | head
