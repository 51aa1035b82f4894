# mask heads: the forward kernel built without SLP vectorization (no packed-f32 VALU beside its MFMAs) vs the in-tree
# build, alternating (tools/mask_heads_bench.py: einsum and the three target sizes)
set -o pipefail
cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out && export TMPDIR=/tmp
L="$GRAFT_REPO_ROOT/tools/lib"
for i in 1 2; do
  timeout -k 10 120 python3 tools/mask_heads_bench.py >> gpurun_out/r5x_mh.txt 2>&1 || exit 1
  timeout -k 10 120 python3 tools/mask_heads_bench.py --lib "$L/libbm2f_mhnoslp.so" >> gpurun_out/r5x_mh.txt 2>&1 || exit 1
done
