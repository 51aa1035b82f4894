set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
for v in 1 0 1; do
M2F_CHANNELS_LAST=$v timeout -k 10 300 python -u bench.py --no-cpu-baseline > gpurun_out/saf_bench$v.log 2>&1 || { tail -30 gpurun_out/saf_bench$v.log; exit 1; }
echo "cl=$v $(tail -1 gpurun_out/saf_bench$v.log | cut -c175-215)"
done
