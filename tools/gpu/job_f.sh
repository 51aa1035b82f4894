# spill fixes (L = 4 at 512 threads / two waves, 32-bit unfused gradient offsets): MSDA tests + A/B vs the HEAD build
set -o pipefail
cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out && export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_msda_gpu.py tests/test_capi.py -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/r5f_tests.log 2>&1 || exit 1
for lv in 3 4; do
  for lib in tools/lib/libbm2f_head.so bm2f_amd/lib/libbm2f.so; do
    echo "== levels $lv lib $lib" >> gpurun_out/r5f_mb.log
    timeout -k 10 120 python -u tools/msda_bench.py --levels $lv --lib $lib >> gpurun_out/r5f_mb.log 2>&1 || exit 1
    timeout -k 10 120 python -u tools/msda_bench.py --levels $lv --fused --lib $lib >> gpurun_out/r5f_mb.log 2>&1 || exit 1
  done
done
