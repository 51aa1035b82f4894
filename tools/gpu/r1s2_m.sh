set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
timeout -k 10 300 python -u -m pytest tests/test_conv_gpu.py -x -q -m gpu --timeout 120 --timeout-method thread > gpurun_out/s2m_tests.log 2>&1; echo "tests rc=$?" >> gpurun_out/s2m_tests.log
timeout -k 10 300 python tools/conv_bench.py > gpurun_out/s2m_bench.log 2>&1
