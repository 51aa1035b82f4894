# round 3, call e: hipBLASLt problem sizes of one config-2 step, kernel traces of config 2 and config 4
set -o pipefail
R=$GRAFT_REPO_ROOT
cd "$R" && mkdir -p gpurun_out && export TMPDIR=/tmp
HIPBLASLT_LOG_MASK=32 HIPBLASLT_LOG_FILE="$R/gpurun_out/hipblaslt_%i.log" timeout -k 10 300 python -u bench.py --steps 1 --warmup 1 \
  --no-cpu-baseline --no-modes --no-peaks --no-dropin --kernel-steps 0 > gpurun_out/blaslt_bench.log 2>&1 && echo "[e] blaslt log ok" && \
timeout -s KILL 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$R/gpurun_out/kt_e2" -o kt -- \
  python3 "$R/bench.py" --steps 3 --warmup 1 --no-cpu-baseline --no-modes --no-peaks --no-dropin --kernel-steps 0 > gpurun_out/kt_e2.log 2>&1 && \
timeout -s KILL 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$R/gpurun_out/kt_e4" -o kt -- \
  python3 "$R/bench.py" --config 4 --steps 5 --warmup 2 --no-peaks --kernel-steps 0 > gpurun_out/kt_e4.log 2>&1 && echo "[e] traces ok"
