set -e
B="timeout -k 10 100 python tools/msda_bench.py --iters 5"
$B --noise 0.3
$B --noise 1.0 --bwd-only
M2F_MSDA_TILE=16 M2F_MSDA_WIN_ROWS=576 $B --noise 0.3 --bwd-only
M2F_MSDA_TILE=10 $B --noise 0.3 --bwd-only
M2F_MSDA_TILE=12 M2F_MSDA_THREADS=512 $B --noise 0.3 --bwd-only
M2F_MSDA_ABLATE=7 $B --noise 0.3 --bwd-only
