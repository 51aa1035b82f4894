set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
timeout -k 10 300 python -u -m pytest tests/test_conv_gpu.py tests/test_modules_gpu.py -x -q --timeout 120 --timeout-method thread > gpurun_out/sab_tests.log 2>&1 || { echo "tests failed"; tail -40 gpurun_out/sab_tests.log; exit 1; }
tail -1 gpurun_out/sab_tests.log
timeout -k 10 200 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/sab_smoke.log 2>&1 || { tail -20 gpurun_out/sab_smoke.log; exit 1; }
tail -1 gpurun_out/sab_smoke.log
for i in 1 2; do
timeout -k 10 300 python -u bench.py --no-cpu-baseline > gpurun_out/sab_bench$i.log 2>&1 || { tail -30 gpurun_out/sab_bench$i.log; exit 1; }
echo "$(tail -1 gpurun_out/sab_bench$i.log | cut -c175-215)"
done
