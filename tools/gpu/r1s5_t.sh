set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
timeout -k 10 200 python -u tools/gemm_x3_bench.py --cfgs 0,4 > gpurun_out/s5t_gemm.log 2>&1 || { tail -20 gpurun_out/s5t_gemm.log; exit 1; }
grep "^fwd" gpurun_out/s5t_gemm.log | sed 's/blas.*x3 /x3 /'
