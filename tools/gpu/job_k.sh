# MSDA backward cell walk: correctness (MSDA tests, config-2 pyramid vs oracle, DET mode), A/B vs the pixel walk,
# cell-row chunk variants; x3 loop A/B vs the HEAD x3 sources; bench
set -o pipefail
cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out && export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_msda_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r5k_tests.log 2>&1 || exit 1
timeout -k 10 600 python -u -m pytest tests/test_scale_gpu.py -m gpu -x -q --timeout 300 --timeout-method thread -k "fused_msda or op_level_dropin" >> gpurun_out/r5k_tests.log 2>&1 || exit 1
for r in 1 2; do
  for lib in tools/lib/libbm2f_pixwalk.so bm2f_amd/lib/libbm2f.so tools/lib/libbm2f_cell2.so tools/lib/libbm2f_cell8.so; do
    for nz in 1.0 4.0; do
      echo "== round $r $lib noise $nz" >> gpurun_out/r5k_mb.log
      timeout -k 10 200 python -u tools/msda_bench.py --fused --bwd-only --noise $nz --lib $lib >> gpurun_out/r5k_mb.log 2>&1 || exit 1
    done
  done
done
for r in 1 2; do
  for lib in tools/lib/libbm2f_x3base.so bm2f_amd/lib/libbm2f.so; do
    echo "== round $r gemm $lib" >> gpurun_out/r5k_x3.log
    timeout -k 10 200 python -u tools/gemm_x3_bench.py --x3-only --cfgs "" --lib $lib >> gpurun_out/r5k_x3.log 2>&1 || exit 1
    echo "== round $r conv $lib" >> gpurun_out/r5k_x3.log
    timeout -k 10 200 python -u tools/conv_bench.py --x3-only --lib $lib >> gpurun_out/r5k_x3.log 2>&1 || exit 1
  done
done
timeout -k 10 300 python -u bench.py --no-modes --no-cpu-baseline --no-dropin > gpurun_out/r5k_bench.json 2> gpurun_out/r5k_bench.err || exit 1
