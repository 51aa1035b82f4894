set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
timeout -k 10 300 python tools/step_breakdown.py > gpurun_out/s2b_breakdown.log 2>&1 && \
timeout -k 10 300 python tools/op_profile.py --rows 60 --attribute > gpurun_out/s2b_opprof.log 2>&1
