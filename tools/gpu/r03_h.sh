# round 3, call h: tests of the changed decoder kernels, add / copy shapes in one fp16 step
set -o pipefail
R=$GRAFT_REPO_ROOT
cd "$R" && mkdir -p gpurun_out && export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_scale_gpu.py tests/test_decoder_gpu.py tests/test_modules_gpu.py \
  tests/test_mask_heads_gpu.py -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/tests_h.log 2>&1 && echo "[h] tests ok" && \
timeout -k 10 300 python -u tools/op_profile.py --rows 5 --shapes aten::add > gpurun_out/op_shapes_add.txt 2>&1 && \
timeout -k 10 300 python -u tools/op_profile.py --rows 5 --shapes aten::copy_ > gpurun_out/op_shapes_copy.txt 2>&1 && echo "[h] shapes ok"
