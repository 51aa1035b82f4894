set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
timeout -k 10 300 python tools/op_profile.py --rows 30 --attribute > gpurun_out/s2e_opprof.log 2>&1
