set -o pipefail
cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out && export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_conv_gpu.py tests/test_capi.py tests/test_modules_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r5d_tests.log 2>&1 || exit 1
timeout -k 10 600 python -u -m pytest tests/test_scale_gpu.py -m gpu -x -q --timeout 300 --timeout-method thread -k "pixdec_config2" > gpurun_out/r5d_tests2.log 2>&1 || exit 1
timeout -k 10 300 python -u bench.py --no-modes --no-cpu-baseline --no-dropin > gpurun_out/r5d_bench.json 2> gpurun_out/r5d_bench.err || exit 1
