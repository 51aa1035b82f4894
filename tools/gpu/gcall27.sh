set -o pipefail
R=$GRAFT_REPO_ROOT
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/prof27 -o run -- python3 $R/bench.py --steps 10 --warmup 3 --no-cpu-baseline > $R/gpurun_out/prof27.log 2>&1 && \
timeout -k 10 400 rocprofv3 --pmc FETCH_SIZE --kernel-include-regex "msda_bwd" --output-format csv -d $R/gpurun_out/pmc27f -o f -- python3 $R/bench.py --steps 2 --warmup 1 --no-cpu-baseline > $R/gpurun_out/pmc27f.log 2>&1 && \
timeout -k 10 400 rocprofv3 --pmc WRITE_SIZE --kernel-include-regex "msda_bwd" --output-format csv -d $R/gpurun_out/pmc27w -o w -- python3 $R/bench.py --steps 2 --warmup 1 --no-cpu-baseline > $R/gpurun_out/pmc27w.log 2>&1
