set -o pipefail
export MIOPEN_USER_DB_PATH=$GRAFT_REPO_ROOT/gpurun_out/miopen_db
mkdir -p $MIOPEN_USER_DB_PATH
export MIOPEN_FIND_MODE=NORMAL
( time timeout -k 10 800 python bench.py --no-cpu-baseline --steps 5 --warmup 2 ) > gpurun_out/bench21_a.json 2> gpurun_out/bench21_a.err && \
( time timeout -k 10 400 python bench.py --no-cpu-baseline --steps 5 --warmup 2 ) > gpurun_out/bench21_b.json 2> gpurun_out/bench21_b.err && \
ls -la $MIOPEN_USER_DB_PATH > gpurun_out/miopen_db_ls.txt
