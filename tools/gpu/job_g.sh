# channels-last R50 backbone: NORMAL-mode MIOpen search for its NHWC convolutions (seeded with the shipped find-db),
# then the bench line in both layouts on the grown db (FAST mode)
set -o pipefail
R=$GRAFT_REPO_ROOT
cd "$R" && mkdir -p gpurun_out/db && export TMPDIR=/tmp
cp bm2f_amd/miopen_db/*.ufdb.txt gpurun_out/db/
( while sleep 45; do echo "[finddb] $(date +%T) db lines: $(cat gpurun_out/db/*.txt | wc -l)"; done ) &
HB=$!
trap 'kill $HB 2>/dev/null' EXIT
MIOPEN_FIND_MODE=NORMAL MIOPEN_USER_DB_PATH="$R/gpurun_out/db" timeout -k 10 800 python -u bench.py --amp fp16 --channels-last 1 \
  --steps 1 --warmup 1 --no-modes --no-cpu-baseline --no-peaks --no-dropin --kernel-steps 0 > gpurun_out/r5g_db_cl.log 2>&1 || exit 1
echo "[finddb] search done"
for cl in 1 0; do
  MIOPEN_USER_DB_PATH="$R/gpurun_out/db" timeout -k 10 300 python -u bench.py --channels-last $cl --no-modes --no-cpu-baseline \
    --no-dropin --no-peaks --kernel-steps 0 > gpurun_out/r5g_bench_cl$cl.json 2> gpurun_out/r5g_bench_cl$cl.err || exit 1
done
