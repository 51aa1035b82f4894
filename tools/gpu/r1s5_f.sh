set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
true

timeout -k 10 120 python -u tools/fpn_bench.py > gpurun_out/s5f_fpn.log 2>&1 || { tail -20 gpurun_out/s5f_fpn.log; exit 1; }
grep -v amdgpu.ids gpurun_out/s5f_fpn.log
timeout -k 10 300 python -u bench.py --no-cpu-baseline > gpurun_out/s5f_bench.log 2>&1 || { tail -30 gpurun_out/s5f_bench.log; exit 1; }
tail -1 gpurun_out/s5f_bench.log | cut -c1-200
