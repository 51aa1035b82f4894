set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
timeout -k 10 400 python -u -m pytest tests -x -q -m gpu --timeout 120 --timeout-method thread > gpurun_out/s2l_tests.log 2>&1; echo "tests rc=$?" >> gpurun_out/s2l_tests.log
timeout -k 10 300 python bench.py > gpurun_out/s2l_bench.json 2> gpurun_out/s2l_bench.err
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/prof_l -o run -- python3 $R/bench.py --steps 10 --warmup 3 --no-cpu-baseline > $R/gpurun_out/prof_l.log 2>&1
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --kernel-include-regex "msda_bwd" --output-format csv -d $R/gpurun_out/pmc_lf -o f -- python3 $R/bench.py --steps 2 --warmup 1 --no-cpu-baseline > $R/gpurun_out/pmc_lf.log 2>&1
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --kernel-include-regex "msda_bwd" --output-format csv -d $R/gpurun_out/pmc_lw -o w -- python3 $R/bench.py --steps 2 --warmup 1 --no-cpu-baseline > $R/gpurun_out/pmc_lw.log 2>&1
