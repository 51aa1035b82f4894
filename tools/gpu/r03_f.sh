# round 3, call f: the full GPU suite + smoke (as the driver runs them), then the default bench line
set -o pipefail
R=$GRAFT_REPO_ROOT
cd "$R" && mkdir -p gpurun_out && export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 200 --timeout-method thread > gpurun_out/tests_f.log 2>&1 && \
echo "[f] tests ok" && \
timeout -k 10 200 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke_f.log 2>&1 && echo "[f] smoke ok" && \
timeout -k 10 500 python -u bench.py > gpurun_out/bench_f.json 2> gpurun_out/bench_f.err && echo "[f] bench ok"
