set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R && mkdir -p gpurun_out
timeout -k 10 120 python -u tools/dbg_msda.py 2>&1 | tee gpurun_out/r2d_dbg.log
