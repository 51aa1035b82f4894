set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
for v in 0 1 0 1; do
M2F_AB_OLD=$v timeout -k 10 300 python -u bench.py --no-cpu-baseline > gpurun_out/s5z_bench$v.log 2>&1 || { tail -30 gpurun_out/s5z_bench$v.log; exit 1; }
echo "old=$v $(tail -1 gpurun_out/s5z_bench$v.log | cut -c175-215)"
done
