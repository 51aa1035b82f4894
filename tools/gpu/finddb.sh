# NORMAL-mode MIOpen search for the bench step's convolutions under AMP fp16 (and bf16 / fp32 entries kept),
# seeded with the shipped find-db, then the bench line on the grown db (FAST mode).
#   gpurun --timeout 1200 -- 'bash tools/gpu/finddb.sh'   -> gpurun_out/db/*.ufdb.txt, gpurun_out/bench.json
set -o pipefail
R=$GRAFT_REPO_ROOT
cd "$R" && mkdir -p gpurun_out/db && export TMPDIR=/tmp
cp bm2f_amd/miopen_db/*.ufdb.txt gpurun_out/db/
( while sleep 45; do echo "[finddb] $(date +%T) db lines: $(cat gpurun_out/db/*.txt | wc -l)"; done ) &
HB=$!
trap 'kill $HB 2>/dev/null' EXIT
MIOPEN_FIND_MODE=NORMAL MIOPEN_USER_DB_PATH="$R/gpurun_out/db" timeout -k 10 700 python -u bench.py --amp fp16 \
  --steps 1 --warmup 1 --no-modes --no-cpu-baseline --no-peaks --kernel-steps 0 > gpurun_out/db_fp16.log 2>&1 && \
echo "[finddb] fp16 search done" && \
MIOPEN_USER_DB_PATH="$R/gpurun_out/db" timeout -k 10 400 python -u bench.py --no-cpu-baseline \
  > gpurun_out/bench.json 2> gpurun_out/bench.err
