set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
true
timeout -k 10 400 python -u bench.py > gpurun_out/s5r2_bench.log 2>&1 || exit 1
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/prof_s5r2 -o run -- python3 $R/bench.py --steps 10 --warmup 3 --no-cpu-baseline > $R/gpurun_out/prof_s5r2.log 2>&1 && \
timeout -k 10 400 rocprofv3 --pmc FETCH_SIZE --kernel-include-regex "msda_bwd" --output-format csv -d $R/gpurun_out/pmc_s5r2f -o f -- python3 $R/bench.py --steps 2 --warmup 1 --no-cpu-baseline > $R/gpurun_out/pmc_s5r2f.log 2>&1 && \
timeout -k 10 400 rocprofv3 --pmc WRITE_SIZE --kernel-include-regex "msda_bwd" --output-format csv -d $R/gpurun_out/pmc_s5r2w -o w -- python3 $R/bench.py --steps 2 --warmup 1 --no-cpu-baseline > $R/gpurun_out/pmc_s5r2w.log 2>&1
rm -f $R/gpurun_out/prof_s5r2/*kernel_trace.csv
