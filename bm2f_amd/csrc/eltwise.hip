// Fused per-channel bias (+ residual) + ReLU over an NCHW activation, in place:
//     y = max(x + r + bias[c], 0)
// NCHW or channels_last (NHWC memory).  For the benchmark's R50 backbone (detectron2 FrozenBatchNorm2d folded into the convs: the conv runs
// without bias and this op applies the BN shift, the residual and the ReLU in one HBM pass instead of
// the library's broadcast bias add, a residual add and a ReLU).  bf16 or fp32, 16-byte vectors; needs
// H*W % 8 == 0 (bf16) / % 4 (fp32) so a vector never straddles two channels.
#include "bm2f.h"
#include "common.h"

#include <hip/hip_runtime.h>

namespace {

template <typename T, int V>
struct Vec {
  T v[V];
};

template <typename T, int V, bool NHWC>
__global__ void __launch_bounds__(256) bias_act_kernel(T* __restrict__ x, const T* __restrict__ r,
                                                       const float* __restrict__ bias, int64_t nvec, int C, int hwv) {
  using VT = Vec<T, V>;
  const int64_t i = blockIdx.x * static_cast<int64_t>(blockDim.x) + threadIdx.x;
  if (i >= nvec) return;
  // NCHW: one channel per vector; NHWC (channels_last): V consecutive channels per vector
  const int c = NHWC ? static_cast<int>((i * V) % C) : static_cast<int>((i / hwv) % C);
  VT a = reinterpret_cast<const VT*>(x)[i];
  VT rr;
  if (r) rr = reinterpret_cast<const VT*>(r)[i];
#pragma unroll
  for (int e = 0; e < V; ++e) {
    float v = static_cast<float>(a.v[e]) + bias[NHWC ? c + e : c];
    if (r) v += static_cast<float>(rr.v[e]);
    a.v[e] = static_cast<T>(fmaxf(v, 0.f));
  }
  reinterpret_cast<VT*>(x)[i] = a;
}

}  // namespace

extern "C" int m2f_bias_act_nchw(void* x, const void* residual, const float* bias, int64_t N, int C, int64_t HW,
                                 int dtype, int channels_last, void* stream) {
  const char* fn = "m2f_bias_act_nchw";
  if (!x || !bias || N < 0 || C <= 0 || HW <= 0) return m2f::fail(M2F_EINVAL, "%s: bad arguments", fn);
  const int V = dtype == M2F_BF16 ? 8 : 4;
  if (dtype != M2F_BF16 && dtype != M2F_F32) return m2f::fail(M2F_EUNSUPPORTED, "%s: dtype %d", fn, dtype);
  if ((channels_last ? C % V : HW % V) || !m2f::aligned(x, 16) || (residual && !m2f::aligned(residual, 16)))
    return m2f::fail(M2F_EUNSUPPORTED, "%s: needs %s %% %d == 0 and 16-byte aligned tensors", fn,
                     channels_last ? "C" : "H*W", V);
  const int64_t nvec = N * C * HW / V;
  if (nvec == 0) return m2f::ok();
  hipStream_t st = static_cast<hipStream_t>(stream);
  const unsigned grid = m2f::ceil_div(nvec, 256);
#define M2F_BA(T, V, L) bias_act_kernel<T, V, L><<<grid, 256, 0, st>>>(static_cast<T*>(x), static_cast<const T*>(residual), \
                                                                      bias, nvec, C, static_cast<int>(HW / V))
  if (dtype == M2F_BF16) {
    if (channels_last) M2F_BA(__bf16, 8, true); else M2F_BA(__bf16, 8, false);
  } else {
    if (channels_last) M2F_BA(float, 4, true); else M2F_BA(float, 4, false);
  }
#undef M2F_BA
  return m2f::check_launch(fn);
}
