# x3 pipeline loops: unconditional pairs (no vmcnt(0) at the loop head) -- correctness, then A/B vs the previous build
set -o pipefail
cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out && export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_linear_gpu.py tests/test_conv_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r5j_tests.log 2>&1 || exit 1
for r in 1 2; do
  for lib in tools/lib/libbm2f_head.so bm2f_amd/lib/libbm2f.so; do
    echo "== round $r gemm $lib" >> gpurun_out/r5j_ab.log
    timeout -k 10 200 python -u tools/gemm_x3_bench.py --x3-only --cfgs "" --lib $lib >> gpurun_out/r5j_ab.log 2>&1 || exit 1
    echo "== round $r conv $lib" >> gpurun_out/r5j_ab.log
    timeout -k 10 200 python -u tools/conv_bench.py --x3-only --lib $lib >> gpurun_out/r5j_ab.log 2>&1 || exit 1
  done
done
timeout -k 10 300 python -u bench.py --no-modes --no-cpu-baseline --no-dropin > gpurun_out/r5j_bench.json 2> gpurun_out/r5j_bench.err || exit 1
