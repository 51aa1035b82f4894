set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
for b in 512 768 1024 1536; do
M2F_GEMM_X3_TN_BLOCKS=$b timeout -k 10 200 python -u tools/gemm_x3_bench.py --cfgs "" > gpurun_out/sac_$b.log 2>&1 || { tail -20 gpurun_out/sac_$b.log; exit 1; }
echo "blocks=$b"; grep "^wgrad" gpurun_out/sac_$b.log | sed 's/blas.*exact_bias[^x]*//' | cut -c1-120
done
