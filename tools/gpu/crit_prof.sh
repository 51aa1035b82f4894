set -o pipefail
R=$GRAFT_REPO_ROOT
cd /tmp && export TMPDIR=/tmp && cd $R
timeout -k 10 400 rocprofv3 --kernel-trace --output-format rocpd -d /tmp/prof_crit -o run -- python3 -u tools/criterion_bench.py --iters 3 > gpurun_out/critp.log 2>&1
python tools/rocpd_stats.py $(find /tmp/prof_crit -name "*.db" | head -1) > gpurun_out/crit_kernel_stats.csv
