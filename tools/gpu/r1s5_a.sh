set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
timeout -k 10 300 python -u tools/op_profile.py --rows 60 --attribute > gpurun_out/s5a_attr.log 2>&1 && \
timeout -k 10 300 python -u tools/op_profile.py --rows 20 --shapes add > gpurun_out/s5a_add.log 2>&1 && \
timeout -k 10 300 python -u tools/op_profile.py --rows 20 --shapes copy_ > gpurun_out/s5a_copy.log 2>&1
