# one-pass memory-gradient sink (m2f_sum_to_f32), channels-last stem max pool: tests, bench, step budget
set -o pipefail
cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out && export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_colsum_gpu.py tests/test_backbone_ops_gpu.py tests/test_modules_gpu.py tests/test_decoder_gpu.py tests/test_capi.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r5m_tests.log 2>&1 || exit 1
timeout -k 10 300 python -u bench.py --no-modes --no-cpu-baseline --no-dropin > gpurun_out/r5m_bench.json 2> gpurun_out/r5m_bench.err || exit 1
timeout -k 10 400 python -u tools/step_budget.py --steps 2 --no-sites --out gpurun_out/r5m_budget > gpurun_out/r5m_budget.log 2>&1 || exit 1
