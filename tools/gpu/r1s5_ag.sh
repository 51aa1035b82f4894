set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
for cfg in "M2F_MSDA_HALO=8" "M2F_MSDA_HALO=6" "M2F_MSDA_HALO=12" "M2F_MSDA_TILE=12" "M2F_MSDA_TILE=20" "M2F_MSDA_THREADS=768"; do
env $cfg timeout -k 10 120 python -u tools/msda_bench.py --bwd-only --iters 10 > gpurun_out/sag.log 2>&1 || { tail -5 gpurun_out/sag.log; continue; }
echo "$cfg: $(grep -o 'bwd [0-9.]* ms' gpurun_out/sag.log | head -1)"
done
