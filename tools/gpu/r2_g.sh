set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R && mkdir -p gpurun_out && export TMPDIR=/tmp
timeout -k 10 120 python -u tools/msda_stamps.py 2>&1 | tee gpurun_out/r2g_stamps.log
