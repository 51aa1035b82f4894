set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
timeout -k 10 300 python -u -m pytest tests/test_conv_gpu.py tests/test_modules_gpu.py -x -q --timeout 120 --timeout-method thread > gpurun_out/sae_tests.log 2>&1 || { echo "tests failed"; tail -40 gpurun_out/sae_tests.log; exit 1; }
tail -1 gpurun_out/sae_tests.log
timeout -k 10 120 python -u tools/fpn_bench.py > gpurun_out/sae_fpn.log 2>&1 || { tail -20 gpurun_out/sae_fpn.log; exit 1; }
grep fused gpurun_out/sae_fpn.log
for i in 1 2; do
timeout -k 10 300 python -u bench.py --no-cpu-baseline > gpurun_out/sae_bench$i.log 2>&1 || { tail -30 gpurun_out/sae_bench$i.log; exit 1; }
echo "$(tail -1 gpurun_out/sae_bench$i.log | cut -c175-215)"
done
