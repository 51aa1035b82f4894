# MSDA forward: the per-level window box reduced by DPP (row steps, row_bcast, readlane) instead of six
# __shfl_xor (ds_bpermute) rounds: MSDA tests, then an alternating A/B of the forward against the previous build
set -o pipefail
cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out && export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_msda_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r5ae_tests.log 2>&1 || exit 1
timeout -k 10 600 python -u -m pytest tests/test_scale_gpu.py -m gpu -x -q --timeout 300 --timeout-method thread -k "fused" >> gpurun_out/r5ae_tests.log 2>&1 || exit 1
B="$GRAFT_REPO_ROOT/tools/lib/libbm2f_base.so"
for i in 1 2; do
  timeout -k 10 120 python3 tools/msda_bench.py --fused --fwd-only --lib "$B" >> gpurun_out/r5ae_mb.txt 2>&1 || exit 1
  timeout -k 10 120 python3 tools/msda_bench.py --fused --fwd-only >> gpurun_out/r5ae_mb.txt 2>&1 || exit 1
  timeout -k 10 120 python3 tools/msda_bench.py --fused --fwd-only --noise 4 --lib "$B" >> gpurun_out/r5ae_mb.txt 2>&1 || exit 1
  timeout -k 10 120 python3 tools/msda_bench.py --fused --fwd-only --noise 4 >> gpurun_out/r5ae_mb.txt 2>&1 || exit 1
  timeout -k 10 120 python3 tools/msda_bench.py --fwd-only --lib "$B" >> gpurun_out/r5ae_mb.txt 2>&1 || exit 1
  timeout -k 10 120 python3 tools/msda_bench.py --fwd-only >> gpurun_out/r5ae_mb.txt 2>&1 || exit 1
done
