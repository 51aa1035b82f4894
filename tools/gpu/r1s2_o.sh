set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
mkdir -p gpurun_out/mdb_cl
cp bm2f_amd/miopen_db/* gpurun_out/mdb_cl/
export MIOPEN_USER_DB_PATH=$R/gpurun_out/mdb_cl
( MIOPEN_FIND_MODE=NORMAL M2F_CHANNELS_LAST=1 timeout -k 10 900 python bench.py --no-cpu-baseline --steps 2 --warmup 1 > gpurun_out/s2o_search.json 2> gpurun_out/s2o_search.err ) && \
( MIOPEN_FIND_MODE=FAST M2F_CHANNELS_LAST=1 timeout -k 10 300 python bench.py --no-cpu-baseline > gpurun_out/s2o_cl.json 2> gpurun_out/s2o_cl.err )
ls -la gpurun_out/mdb_cl
