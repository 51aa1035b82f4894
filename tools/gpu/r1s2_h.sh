set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
M2F_GEMM_X3_TN_NW=4 timeout -k 10 300 python tools/gemm_x3_bench.py --cfgs "" 2>&1 | grep "N1=288" > gpurun_out/s2h_tn.log
timeout -k 10 300 python bench.py --no-cpu-baseline > gpurun_out/s2h_bench.json 2> gpurun_out/s2h_bench.err
M2F_GEMM_X3_TN_NW=4 timeout -k 10 300 python bench.py --no-cpu-baseline > gpurun_out/s2h_bench4.json 2> gpurun_out/s2h_bench4.err
