set -o pipefail
mkdir -p $GRAFT_REPO_ROOT/gpurun_out/mdb23
cp $GRAFT_REPO_ROOT/bm2f_amd/miopen_db/* $GRAFT_REPO_ROOT/gpurun_out/mdb23/
export MIOPEN_USER_DB_PATH=$GRAFT_REPO_ROOT/gpurun_out/mdb23
export MIOPEN_FIND_MODE=FAST
( time timeout -k 10 400 python bench.py --no-cpu-baseline --steps 5 --warmup 2 ) > gpurun_out/bench23.json 2> gpurun_out/bench23.err && \
timeout -k 10 300 python tools/step_breakdown.py > gpurun_out/brk23.log 2>&1
