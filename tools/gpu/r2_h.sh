set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R && mkdir -p gpurun_out && export TMPDIR=/tmp
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_INSTS_VALU SQ_INSTS_LDS SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU GRBM_GUI_ACTIVE --kernel-include-regex msda_bwd --output-format csv -d $R/gpurun_out/r2h_sq -o sq -- python3 $R/tools/msda_bench.py --bwd-only --iters 3 > gpurun_out/r2h_sq.log 2>&1
echo "sq rc=$?"
timeout -s KILL 120 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_VMEM SQ_INSTS_SALU SQ_WAIT_INST_LDS SQ_ACTIVE_INST_LDS SQ_INST_CYCLES_VMEM SQ_ACTIVE_INST_SCA GRBM_GUI_ACTIVE --kernel-include-regex msda_bwd --output-format csv -d $R/gpurun_out/r2h_lds -o lds -- python3 $R/tools/msda_bench.py --bwd-only --iters 3 > gpurun_out/r2h_lds.log 2>&1
echo "lds rc=$?"
