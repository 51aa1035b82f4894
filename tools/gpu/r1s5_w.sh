set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
timeout -k 10 300 python -u tools/op_profile.py --rows 40 --attribute > gpurun_out/s5w_attr.log 2>&1
