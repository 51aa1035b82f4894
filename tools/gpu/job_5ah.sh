# x3 NT GEMM: 96-wide columns of 8 waves (x3_nt_cfg 4) against 4 waves (cfg 1, the N = 3 * 96k default) and the
# 128-wide configs, encoder-layer shapes (tools/gemm_x3_bench.py --x3-only), twice
set -o pipefail
cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out && export TMPDIR=/tmp
for i in 1 2; do
  timeout -k 10 300 python3 tools/gemm_x3_bench.py --x3-only --cfgs 1,4,3 >> gpurun_out/r5ah_gemm.txt 2>&1 || exit 1
done
