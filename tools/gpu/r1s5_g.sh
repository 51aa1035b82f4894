set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
true

timeout -k 10 120 python -u tools/fpn_bench.py > gpurun_out/s5g_fpn.log 2>&1 || { tail -20 gpurun_out/s5g_fpn.log; exit 1; }
grep -v amdgpu.ids gpurun_out/s5g_fpn.log
true

