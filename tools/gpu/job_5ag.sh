# MSDA backward: the work queue's unit index read by v_readlane (not a ds_bpermute round trip per unit): MSDA tests,
# then an alternating A/B of the fused backward against the previous build (near-init and N(0, 4 px) offsets)
set -o pipefail
cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out && export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_msda_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r5ag_tests.log 2>&1 || exit 1
timeout -k 10 600 python -u -m pytest tests/test_scale_gpu.py -m gpu -x -q --timeout 300 --timeout-method thread -k "fused" >> gpurun_out/r5ag_tests.log 2>&1 || exit 1
B="$GRAFT_REPO_ROOT/tools/lib/libbm2f_base.so"
for i in 1 2; do
  timeout -k 10 120 python3 tools/msda_bench.py --fused --bwd-only --lib "$B" >> gpurun_out/r5ag_mb.txt 2>&1 || exit 1
  timeout -k 10 120 python3 tools/msda_bench.py --fused --bwd-only >> gpurun_out/r5ag_mb.txt 2>&1 || exit 1
  timeout -k 10 120 python3 tools/msda_bench.py --fused --bwd-only --noise 4 --lib "$B" >> gpurun_out/r5ag_mb.txt 2>&1 || exit 1
  timeout -k 10 120 python3 tools/msda_bench.py --fused --bwd-only --noise 4 >> gpurun_out/r5ag_mb.txt 2>&1 || exit 1
done
