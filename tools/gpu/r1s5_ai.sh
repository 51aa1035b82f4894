set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/sai_tests.log 2>&1 || { echo "tests failed"; tail -40 gpurun_out/sai_tests.log; exit 1; }
tail -1 gpurun_out/sai_tests.log
timeout -k 10 200 python -u -c "import __graft_entry__ as g; g.smoke()" 2>&1 | tail -1
