# One rocprofv3 --pmc pass per counter set over a command, each its own run (gpurun rules: no trace domains beside
# --pmc, at most 8 SQ / 4 TCC / 2 TA / 2 TD / 2 GRBM counters per pass), summaries per kernel.
#   PMC_TAG=name PMC_CMD="python3 tools/msda_bench.py --fused --fwd-only --iters 3" bash tools/gpu/pmc_pass.sh SET...
# SET: issue | wait | lds | ta | fetch | write | mfma | coexec
set -o pipefail
R=$GRAFT_REPO_ROOT
cd "$R" && mkdir -p gpurun_out && export TMPDIR=/tmp
declare -A C=(
  [issue]="SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_SALU SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE"
  [wait]="SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VMEM GRBM_GUI_ACTIVE"
  [lds]="SQ_WAIT_INST_LDS SQ_ACTIVE_INST_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_LDS SQ_ACTIVE_INST_ANY SQ_WAVE_CYCLES GRBM_GUI_ACTIVE"
  [ta]="TA_TA_BUSY_sum TA_BUFFER_READ_WAVEFRONTS_sum GRBM_GUI_ACTIVE"
  [fetch]="FETCH_SIZE GRBM_GUI_ACTIVE"
  [write]="WRITE_SIZE GRBM_GUI_ACTIVE"
  [mfma]="SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VALU_MFMA_MOPS_BF16 SQ_INSTS_VALU_MFMA_MOPS_F16 SQ_INSTS_VALU_MFMA_MOPS_F32 GRBM_GUI_ACTIVE"
  [coexec]="SQ_VALU_MFMA_BUSY_CYCLES SQ_VALU_MFMA_COEXEC_CYCLES SQ_INSTS_MFMA SQ_INSTS_VALU SQ_WAIT_INST_LDS SQ_INST_LEVEL_LDS SQ_WAVE_CYCLES GRBM_GUI_ACTIVE"
)
for s in "$@"; do
  d="gpurun_out/pmc_${PMC_TAG}_$s"
  timeout -s KILL 120 rocprofv3 --pmc ${C[$s]} --output-format csv -d "$R/$d" -o p -- $PMC_CMD > "$d.log" 2>&1 || exit 1
  python3 tools/pmc_summary.py $(find "$R/$d" -name "*counter_collection.csv") --top 12 --all > "$d.txt" 2>&1 || exit 1
done
