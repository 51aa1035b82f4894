set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
for cfg in "M2F_MSDA_HALO=4" "M2F_MSDA_HALO=5" "M2F_MSDA_HALO=6" "M2F_MSDA_HALO=7" "M2F_MSDA_HALO=8"; do
env $cfg timeout -k 10 120 python -u tools/msda_bench.py --bwd-only --iters 10 > gpurun_out/sah.log 2>&1 || { tail -5 gpurun_out/sah.log; continue; }
echo "$cfg: $(grep -o 'bwd [0-9.]* ms' gpurun_out/sah.log | head -1)"
done
for cfg in "M2F_MSDA_HALO=6" "M2F_MSDA_HALO=8" "M2F_MSDA_HALO=6" "M2F_MSDA_HALO=8"; do
env $cfg timeout -k 10 300 python -u bench.py --no-cpu-baseline > gpurun_out/sah_b.log 2>&1 || { tail -5 gpurun_out/sah_b.log; exit 1; }
python -c "import json; d=json.loads(open('gpurun_out/sah_b.log').read().strip().splitlines()[-1]); print('$cfg', d['ms_per_step'], d['kernels']['msda_bwd']['mean_ms'])"
done
