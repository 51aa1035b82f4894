set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
timeout -k 10 300 python -u -m pytest tests/test_linear_gpu.py -x -q --timeout 120 --timeout-method thread > gpurun_out/sad_tests.log 2>&1 || { echo "tests failed"; tail -40 gpurun_out/sad_tests.log; exit 1; }
tail -1 gpurun_out/sad_tests.log
timeout -k 10 200 python -u tools/gemm_x3_bench.py --cfgs "" > gpurun_out/sad_gemm.log 2>&1 || { tail -20 gpurun_out/sad_gemm.log; exit 1; }
grep "^wgrad" gpurun_out/sad_gemm.log | sed 's/blas.*exact_bias[^x]*//' | cut -c1-80
for i in 1 2; do
timeout -k 10 300 python -u bench.py --no-cpu-baseline > gpurun_out/sad_bench$i.log 2>&1 || { tail -30 gpurun_out/sad_bench$i.log; exit 1; }
echo "$(tail -1 gpurun_out/sad_bench$i.log | cut -c175-215)"
done
