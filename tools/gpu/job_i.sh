# 16-bit backbone features read directly by the 1x1 x3 convs: bitwise tests, module tests, bench + step budget (channels-last)
set -o pipefail
cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out && export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_conv_gpu.py tests/test_modules_gpu.py tests/test_capi.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r5i_tests.log 2>&1 || exit 1
timeout -k 10 300 python -u bench.py --no-modes --no-cpu-baseline --no-dropin > gpurun_out/r5i_bench.json 2> gpurun_out/r5i_bench.err || exit 1
timeout -k 10 400 python -u tools/step_budget.py --steps 2 --no-sites --out gpurun_out/r5i_budget > gpurun_out/r5i_budget.log 2>&1 || exit 1
