set -o pipefail
mkdir -p $GRAFT_REPO_ROOT/gpurun_out/mdb $GRAFT_REPO_ROOT/gpurun_out/mcache
cp $GRAFT_REPO_ROOT/bm2f_amd/miopen_db/* $GRAFT_REPO_ROOT/gpurun_out/mdb/
export MIOPEN_USER_DB_PATH=$GRAFT_REPO_ROOT/gpurun_out/mdb
export MIOPEN_CUSTOM_CACHE_DIR=$GRAFT_REPO_ROOT/gpurun_out/mcache
export MIOPEN_FIND_MODE=NORMAL
( time timeout -k 10 800 python bench.py --no-cpu-baseline --steps 5 --warmup 2 ) > gpurun_out/bench22_a.json 2> gpurun_out/bench22_a.err && \
( time timeout -k 10 400 python bench.py --no-cpu-baseline --steps 5 --warmup 2 ) > gpurun_out/bench22_b.json 2> gpurun_out/bench22_b.err && \
ls -laR $GRAFT_REPO_ROOT/gpurun_out/mcache $GRAFT_REPO_ROOT/gpurun_out/mdb > gpurun_out/miopen_ls22.txt
