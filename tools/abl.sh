set -e
B="timeout -k 10 100 python tools/msda_bench.py --iters 5 --bwd-only"
for noise in 0.0 0.3 1.0; do $B --noise $noise; done
for ab in 1 2 4 7; do M2F_MSDA_ABLATE=$ab $B --noise 1.0; done
M2F_MSDA_ABLATE=7 $B --noise 0.0
M2F_MSDA_BWD_TILED=0 $B --noise 0.0
