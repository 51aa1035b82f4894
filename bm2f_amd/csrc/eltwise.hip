// Fused per-channel bias (+ residual) + ReLU over an NCHW activation, in place:
//     y = max(x + r + bias[c], 0)
// NCHW or channels_last (NHWC memory).  For the benchmark's R50 backbone (detectron2 FrozenBatchNorm2d folded into the convs: the conv runs
// without bias and this op applies the BN shift, the residual and the ReLU in one HBM pass instead of
// the library's broadcast bias add, a residual add and a ReLU).  bf16, fp16 or fp32, 16-byte vectors; needs
// H*W % 8 == 0 (bf16 / fp16) / % 4 (fp32) so a vector never straddles two channels.
#include "bm2f.h"
#include "common.h"

#include <hip/hip_runtime.h>

#include <algorithm>
#include <mutex>
#include <set>
#include <tuple>

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
    a.v[e] = static_cast<T>(v > 0.f || v != v ? v : 0.f);   // torch's relu: NaN propagates
  }
  reinterpret_cast<VT*>(x)[i] = a;
}

}  // namespace

extern "C" int m2f_bias_act_nchw(void* x, const void* residual, const float* bias, int64_t N, int C, int64_t HW,
                                 int dtype, int channels_last, void* stream) {
  const char* fn = "m2f_bias_act_nchw";
  if (!x || !bias || N < 0 || C <= 0 || HW <= 0) return m2f::fail(M2F_EINVAL, "%s: bad arguments", fn);
  if (dtype != M2F_BF16 && dtype != M2F_F16 && dtype != M2F_F32)
    return m2f::fail(M2F_EUNSUPPORTED, "%s: dtype %d", fn, dtype);
  const int V = dtype == M2F_F32 ? 4 : 8;
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
  } else if (dtype == M2F_F16) {
    if (channels_last) M2F_BA(_Float16, 8, true); else M2F_BA(_Float16, 8, false);
  } else {
    if (channels_last) M2F_BA(float, 4, true); else M2F_BA(float, 4, false);
  }
#undef M2F_BA
  return m2f::check_launch(fn);
}

// ---------------------------------------------------------------------------------------------------
// ReLU backward over the gradients of several consumers of one activation (a residual block's output feeds
// the next block's first conv, its shortcut / identity path and, at a stage end, the pixel decoder):
//     out = (g_0 + ... + g_{k-1}) masked where y <= 0 (torch's threshold_backward rule: a NaN y passes)
// one pass (k + 1 reads, one write) instead of the autograd engine's k - 1 accumulating adds and a separate
// threshold_backward.  The sum is formed in fp32 in consumer order and rounded once.
// ---------------------------------------------------------------------------------------------------
namespace {

constexpr int kMaxReluGrads = 4;

struct ReluGrads {
  const void* g[kMaxReluGrads];
};

template <typename T, int V>
__global__ void __launch_bounds__(256) relu_bwd_sum_kernel(ReluGrads gs, int ng, const T* __restrict__ y,
                                                           T* __restrict__ out, int64_t nvec) {
  using VT = Vec<T, V>;
  const int64_t i = blockIdx.x * static_cast<int64_t>(blockDim.x) + threadIdx.x;
  if (i >= nvec) return;
  float acc[V];
  const VT g0 = reinterpret_cast<const VT*>(gs.g[0])[i];
#pragma unroll
  for (int e = 0; e < V; ++e) acc[e] = static_cast<float>(g0.v[e]);
  for (int k = 1; k < ng; ++k) {
    const VT gk = reinterpret_cast<const VT*>(gs.g[k])[i];
#pragma unroll
    for (int e = 0; e < V; ++e) acc[e] += static_cast<float>(gk.v[e]);
  }
  const VT yy = reinterpret_cast<const VT*>(y)[i];
  VT o;
#pragma unroll
  for (int e = 0; e < V; ++e) o.v[e] = static_cast<T>(!(static_cast<float>(yy.v[e]) <= 0.f) ? acc[e] : 0.f);  // threshold_backward: NaN y passes
  reinterpret_cast<VT*>(out)[i] = o;
}

}  // namespace

extern "C" int m2f_relu_bwd_sum(const void* const* grads, int ngrads, const void* y, void* out, int64_t n, int dtype,
                                void* stream) {
  const char* fn = "m2f_relu_bwd_sum";
  if (!grads || ngrads < 1 || ngrads > kMaxReluGrads || !y || !out || n < 0)
    return m2f::fail(M2F_EINVAL, "%s: bad arguments (1 <= grads <= %d)", fn, kMaxReluGrads);
  if (dtype != M2F_BF16 && dtype != M2F_F16 && dtype != M2F_F32)
    return m2f::fail(M2F_EUNSUPPORTED, "%s: dtype %d", fn, dtype);
  const int V = dtype == M2F_F32 ? 4 : 8;
  ReluGrads gs{};
  bool aligned = m2f::aligned(y, 16) && m2f::aligned(out, 16);
  for (int k = 0; k < ngrads; ++k) {
    if (!grads[k]) return m2f::fail(M2F_EINVAL, "%s: null gradient %d", fn, k);
    gs.g[k] = grads[k];
    aligned = aligned && m2f::aligned(grads[k], 16);
  }
  if (n % V || !aligned) return m2f::fail(M2F_EUNSUPPORTED, "%s: needs n %% %d == 0 and 16-byte aligned tensors", fn, V);
  const int64_t nvec = n / V;
  if (nvec == 0) return m2f::ok();
  hipStream_t st = static_cast<hipStream_t>(stream);
  const unsigned grid = m2f::ceil_div(nvec, 256);
  if (dtype == M2F_BF16)
    relu_bwd_sum_kernel<__bf16, 8><<<grid, 256, 0, st>>>(gs, ngrads, static_cast<const __bf16*>(y),
                                                         static_cast<__bf16*>(out), nvec);
  else if (dtype == M2F_F16)
    relu_bwd_sum_kernel<_Float16, 8><<<grid, 256, 0, st>>>(gs, ngrads, static_cast<const _Float16*>(y),
                                                           static_cast<_Float16*>(out), nvec);
  else
    relu_bwd_sum_kernel<float, 4><<<grid, 256, 0, st>>>(gs, ngrads, static_cast<const float*>(y),
                                                        static_cast<float*>(out), nvec);
  return m2f::check_launch(fn);
}

// ---------------------------------------------------------------------------------------------------
// The fp32 sum of k same-shaped low-precision (or fp32) tensors, in order: out = ((s_0 + s_1) + ...) + s_{k-1}
// with every term converted to fp32 and every add an fp32 add -- the values of out = s_0.float() followed by
// k - 1 in-place `out += s_i` (torch's mixed-dtype add), in one pass (k reads, one write) instead of k.  The
// decoder's memory-token input gradients: one per K / V projection of every layer reading a level
// (mask2former_transformer_decoder.py:103-108), summed in fp32 as autograd sums the cast backward's results.
// ---------------------------------------------------------------------------------------------------
namespace {

constexpr int kMaxSumTerms = 8;

struct SumTerms {
  const void* s[kMaxSumTerms];
};

template <typename T, int V>
__global__ void __launch_bounds__(256) sum_to_f32_kernel(SumTerms ts, int k, float* __restrict__ out, int64_t nvec) {
  using VT = Vec<T, V>;
  const int64_t i = blockIdx.x * static_cast<int64_t>(blockDim.x) + threadIdx.x;
  if (i >= nvec) return;
  float acc[V];
  const VT s0 = reinterpret_cast<const VT*>(ts.s[0])[i];
#pragma unroll
  for (int e = 0; e < V; ++e) acc[e] = static_cast<float>(s0.v[e]);
  for (int t = 1; t < k; ++t) {
    const VT st = reinterpret_cast<const VT*>(ts.s[t])[i];
#pragma unroll
    for (int e = 0; e < V; ++e) acc[e] += static_cast<float>(st.v[e]);
  }
#pragma unroll
  for (int e = 0; e < V; e += 4)
    *reinterpret_cast<float4*>(out + i * V + e) = make_float4(acc[e], acc[e + 1], acc[e + 2], acc[e + 3]);
}

}  // namespace

extern "C" int m2f_sum_to_f32(const void* const* srcs, int k, int64_t n, int dtype, float* out, void* stream) {
  const char* fn = "m2f_sum_to_f32";
  if (!srcs || k < 1 || k > kMaxSumTerms || !out || n < 0)
    return m2f::fail(M2F_EINVAL, "%s: bad arguments (1 <= terms <= %d)", fn, kMaxSumTerms);
  if (dtype != M2F_BF16 && dtype != M2F_F16 && dtype != M2F_F32)
    return m2f::fail(M2F_EUNSUPPORTED, "%s: dtype %d", fn, dtype);
  const int V = 8;
  SumTerms ts{};
  bool aligned = m2f::aligned(out, 16);
  for (int t = 0; t < k; ++t) {
    if (!srcs[t]) return m2f::fail(M2F_EINVAL, "%s: null term %d", fn, t);
    ts.s[t] = srcs[t];
    aligned = aligned && m2f::aligned(srcs[t], 16);
  }
  if (n % V || !aligned) return m2f::fail(M2F_EUNSUPPORTED, "%s: needs n %% %d == 0 and 16-byte aligned tensors", fn, V);
  const int64_t nvec = n / V;
  if (nvec == 0) return m2f::ok();
  hipStream_t st = static_cast<hipStream_t>(stream);
  const unsigned grid = m2f::ceil_div(nvec, 256);
  if (dtype == M2F_BF16) sum_to_f32_kernel<__bf16, 8><<<grid, 256, 0, st>>>(ts, k, out, nvec);
  else if (dtype == M2F_F16) sum_to_f32_kernel<_Float16, 8><<<grid, 256, 0, st>>>(ts, k, out, nvec);
  else sum_to_f32_kernel<float, 8><<<grid, 256, 0, st>>>(ts, k, out, nvec);
  return m2f::check_launch(fn);
}

// ---------------------------------------------------------------------------------------------------
// The benchmark backbone's stem max pool, kernel 3, stride 2, padding 1 (detectron2 BasicStem), NCHW.
// Forward: torch's max_pool2d_with_indices rule (first maximum in window order, NaN wins), the winner
// kept as a 1-byte window position (0..8) instead of an int64 flat index.  Backward: each input pixel
// gathers the gradients of the <= 2 x 2 windows whose winner it is, in torch's (ph, pw) order with an fp32
// sum -- the same arithmetic as max_pool_backward_nchw, on 1/8 of its index bytes.
// ---------------------------------------------------------------------------------------------------
namespace {

template <typename T>
__global__ void __launch_bounds__(256) maxpool3s2_fwd(const T* __restrict__ x, T* __restrict__ y,
                                                     uint8_t* __restrict__ win, int H, int W, int OH, int OW,
                                                     int64_t total) {
  const int64_t t = blockIdx.x * static_cast<int64_t>(blockDim.x) + threadIdx.x;
  if (t >= total) return;
  const int ow = static_cast<int>(t % OW);
  const int64_t r = t / OW;
  const int oh = static_cast<int>(r % OH);
  const int64_t plane = r / OH;
  const T* xp = x + plane * H * W;
  const int h0 = 2 * oh - 1, w0 = 2 * ow - 1;
  const int hs = max(h0, 0), he = min(h0 + 3, H), ws = max(w0, 0), we = min(w0 + 3, W);
  float best = -INFINITY;
  int bi = (hs - h0) * 3 + (ws - w0);
  for (int h = hs; h < he; ++h)
    for (int w = ws; w < we; ++w) {
      const float v = static_cast<float>(xp[h * W + w]);
      if (v > best || v != v) {
        best = v;
        bi = (h - h0) * 3 + (w - w0);
      }
    }
  y[t] = static_cast<T>(best);
  win[t] = static_cast<uint8_t>(bi);
}

template <typename T>
__global__ void __launch_bounds__(256) maxpool3s2_bwd(const T* __restrict__ gy, const uint8_t* __restrict__ win,
                                                     T* __restrict__ gx, int H, int W, int OH, int OW,
                                                     int64_t total) {
  const int64_t t = blockIdx.x * static_cast<int64_t>(blockDim.x) + threadIdx.x;
  if (t >= total) return;
  const int w = static_cast<int>(t % W);
  const int64_t r = t / W;
  const int h = static_cast<int>(r % H);
  const int64_t plane = r / H;
  // windows ph with 2 ph - 1 <= h <= 2 ph + 1 (torch: phstart = h + 1 < 3 ? 0 : (h + 1 - 3) / 2 + 1)
  const int phs = h + 1 < 3 ? 0 : (h - 2) / 2 + 1, phe = min((h + 1) / 2 + 1, OH);
  const int pws = w + 1 < 3 ? 0 : (w - 2) / 2 + 1, pwe = min((w + 1) / 2 + 1, OW);
  const T* gp = gy + plane * OH * OW;
  const uint8_t* wp = win + plane * OH * OW;
  float acc = 0.f;
  for (int ph = phs; ph < phe; ++ph)
    for (int pw = pws; pw < pwe; ++pw) {
      const int o = ph * OW + pw;
      if (wp[o] == (h - (2 * ph - 1)) * 3 + (w - (2 * pw - 1))) acc += static_cast<float>(gp[o]);
    }
  gx[t] = static_cast<T>(acc);
}

// 8 consecutive input pixels of one row per thread (W % 8 == 0): the <= 2 x 6 covering windows' gradients
// and winner bytes are loaded once into registers, the 8 results leave as one 16-byte store
template <typename T>
__global__ void __launch_bounds__(256) maxpool3s2_bwd8(const T* __restrict__ gy, const uint8_t* __restrict__ win,
                                                      T* __restrict__ gx, int H, int W, int OH, int OW,
                                                      int64_t total8) {
  const int64_t t = blockIdx.x * static_cast<int64_t>(blockDim.x) + threadIdx.x;
  if (t >= total8) return;
  const int W8 = W / 8;
  const int w0 = static_cast<int>(t % W8) * 8;
  const int64_t r = t / W8;
  const int h = static_cast<int>(r % H);
  const int64_t plane = r / H;
  const int phs = h + 1 < 3 ? 0 : (h - 2) / 2 + 1, phe = min((h + 1) / 2 + 1, OH);
  const int pwb = w0 + 1 < 3 ? 0 : (w0 - 2) / 2 + 1;   // first window column any of the 8 pixels touches
  const T* gp = gy + plane * OH * OW;
  const uint8_t* wp = win + plane * OH * OW;
  float g[2][6];
  int wi[2][6];
#pragma unroll
  for (int a = 0; a < 2; ++a)
#pragma unroll
    for (int b = 0; b < 6; ++b) {
      const int ph = phs + a, pw = pwb + b;
      const bool in = ph < phe && pw < OW;
      const int o = in ? ph * OW + pw : 0;
      g[a][b] = in ? static_cast<float>(gp[o]) : 0.f;
      wi[a][b] = in ? static_cast<int>(wp[o]) : -1;
    }
  T res[8];
#pragma unroll
  for (int e = 0; e < 8; ++e) {
    const int w = w0 + e;
    const int pws = w + 1 < 3 ? 0 : (w - 2) / 2 + 1, pwe = min((w + 1) / 2 + 1, OW);
    float acc = 0.f;
#pragma unroll
    for (int a = 0; a < 2; ++a)
#pragma unroll
      for (int b = 0; b < 6; ++b) {
        const int ph = phs + a, pw = pwb + b;
        // torch's order: ph outer, pw inner, over [phs, phe) x [pws, pwe)
        if (ph < phe && pw >= pws && pw < pwe && wi[a][b] == (h - (2 * ph - 1)) * 3 + (w - (2 * pw - 1)))
          acc += g[a][b];
      }
    res[e] = static_cast<T>(acc);
  }
  T* dst = gx + (plane * H + h) * static_cast<int64_t>(W) + w0;
  if constexpr (sizeof(T) == 2) {
    *reinterpret_cast<uint4*>(dst) = *reinterpret_cast<const uint4*>(res);
  } else {
    reinterpret_cast<uint4*>(dst)[0] = reinterpret_cast<const uint4*>(res)[0];
    reinterpret_cast<uint4*>(dst)[1] = reinterpret_cast<const uint4*>(res)[1];
  }
}

// NHWC (channels-last) forms: a thread per (pixel, 8 channels), every window read as 16-byte channel vectors; the
// same per-channel rules and order as the NCHW kernels above (first maximum in window order, a NaN wins; the
// backward's (ph, pw) order with an fp32 sum).  C % 8 == 0.
template <typename T>
__global__ void __launch_bounds__(256) maxpool3s2_fwd_nhwc(const T* __restrict__ x, T* __restrict__ y,
                                                          uint8_t* __restrict__ win, int H, int W, int OH, int OW,
                                                          int C, int64_t total8) {
  using VT = Vec<T, 8>;
  const int64_t t = blockIdx.x * static_cast<int64_t>(blockDim.x) + threadIdx.x;
  if (t >= total8) return;
  const int C8 = C / 8;
  const int c8 = static_cast<int>(t % C8);
  int64_t r = t / C8;
  const int ow = static_cast<int>(r % OW);
  r /= OW;
  const int oh = static_cast<int>(r % OH);
  const int64_t n = r / OH;
  const int h0 = 2 * oh - 1, w0 = 2 * ow - 1;
  const int hs = max(h0, 0), he = min(h0 + 3, H), ws = max(w0, 0), we = min(w0 + 3, W);
  float best[8];
  int bi[8];
#pragma unroll
  for (int e = 0; e < 8; ++e) {
    best[e] = -INFINITY;
    bi[e] = (hs - h0) * 3 + (ws - w0);
  }
  const T* xp = x + (n * H * W) * C + c8 * 8;
  for (int h = hs; h < he; ++h)
    for (int w = ws; w < we; ++w) {
      const VT v = *reinterpret_cast<const VT*>(xp + (static_cast<int64_t>(h) * W + w) * C);
      const int k = (h - h0) * 3 + (w - w0);
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        const float f = static_cast<float>(v.v[e]);
        if (f > best[e] || f != f) {
          best[e] = f;
          bi[e] = k;
        }
      }
    }
  VT o;
  uint8_t wb[8];
#pragma unroll
  for (int e = 0; e < 8; ++e) {
    o.v[e] = static_cast<T>(best[e]);
    wb[e] = static_cast<uint8_t>(bi[e]);
  }
  const int64_t oo = ((n * OH + oh) * OW + ow) * C + c8 * 8;
  *reinterpret_cast<VT*>(y + oo) = o;
  *reinterpret_cast<uint2*>(win + oo) = *reinterpret_cast<const uint2*>(wb);
}

template <typename T>
__global__ void __launch_bounds__(256) maxpool3s2_bwd_nhwc(const T* __restrict__ gy, const uint8_t* __restrict__ win,
                                                          T* __restrict__ gx, int H, int W, int OH, int OW, int C,
                                                          int64_t total8) {
  using VT = Vec<T, 8>;
  const int64_t t = blockIdx.x * static_cast<int64_t>(blockDim.x) + threadIdx.x;
  if (t >= total8) return;
  const int C8 = C / 8;
  const int c8 = static_cast<int>(t % C8);
  int64_t r = t / C8;
  const int w = static_cast<int>(r % W);
  r /= W;
  const int h = static_cast<int>(r % H);
  const int64_t n = r / H;
  const int phs = h + 1 < 3 ? 0 : (h - 2) / 2 + 1, phe = min((h + 1) / 2 + 1, OH);
  const int pws = w + 1 < 3 ? 0 : (w - 2) / 2 + 1, pwe = min((w + 1) / 2 + 1, OW);
  float acc[8];
#pragma unroll
  for (int e = 0; e < 8; ++e) acc[e] = 0.f;
  for (int ph = phs; ph < phe; ++ph)
    for (int pw = pws; pw < pwe; ++pw) {
      const int64_t o = ((n * OH + ph) * OW + pw) * C + c8 * 8;
      const VT g = *reinterpret_cast<const VT*>(gy + o);
      uint8_t wb[8];
      *reinterpret_cast<uint2*>(wb) = *reinterpret_cast<const uint2*>(win + o);
      const int k = (h - (2 * ph - 1)) * 3 + (w - (2 * pw - 1));
#pragma unroll
      for (int e = 0; e < 8; ++e)
        if (wb[e] == k) acc[e] += static_cast<float>(g.v[e]);
    }
  VT o;
#pragma unroll
  for (int e = 0; e < 8; ++e) o.v[e] = static_cast<T>(acc[e]);
  *reinterpret_cast<VT*>(gx + ((n * H + h) * W + w) * C + c8 * 8) = o;
}

}  // namespace

extern "C" int m2f_maxpool3s2_nhwc(int backward, const void* src, void* dst, uint8_t* window, int N, int H, int W,
                                   int C, int dtype, void* stream) {
  const char* fn = "m2f_maxpool3s2_nhwc";
  if (!src || !dst || !window || N < 0 || H <= 0 || W <= 0 || C <= 0) return m2f::fail(M2F_EINVAL, "%s: bad arguments", fn);
  if (dtype != M2F_BF16 && dtype != M2F_F16) return m2f::fail(M2F_EUNSUPPORTED, "%s: dtype %d (16-bit only)", fn, dtype);
  if (C % 8 || !m2f::aligned(src, 16) || !m2f::aligned(dst, 16) || !m2f::aligned(window, 8))
    return m2f::fail(M2F_EUNSUPPORTED, "%s: needs C %% 8 == 0 and aligned tensors", fn);
  const int OH = (H - 1) / 2 + 1, OW = (W - 1) / 2 + 1;
  const int64_t total8 = static_cast<int64_t>(N) * (backward ? static_cast<int64_t>(H) * W : static_cast<int64_t>(OH) * OW) * (C / 8);
  if (total8 == 0) return m2f::ok();
  hipStream_t st = static_cast<hipStream_t>(stream);
  const unsigned grid = m2f::ceil_div(total8, 256);
#define M2F_MPN(T)                                                                                                     \
  if (backward)                                                                                                        \
    maxpool3s2_bwd_nhwc<T><<<grid, 256, 0, st>>>(static_cast<const T*>(src), window, static_cast<T*>(dst), H, W, OH,   \
                                                 OW, C, total8);                                                       \
  else                                                                                                                 \
    maxpool3s2_fwd_nhwc<T><<<grid, 256, 0, st>>>(static_cast<const T*>(src), static_cast<T*>(dst), window, H, W, OH,   \
                                                 OW, C, total8);
  if (dtype == M2F_BF16) { M2F_MPN(__bf16) } else { M2F_MPN(_Float16) }
#undef M2F_MPN
  return m2f::check_launch(fn);
}

extern "C" int m2f_maxpool3s2_fwd(const void* x, void* y, uint8_t* window, int64_t planes, int H, int W, int dtype,
                                  void* stream) {
  const char* fn = "m2f_maxpool3s2_fwd";
  if (!x || !y || !window || planes < 0 || H <= 0 || W <= 0) return m2f::fail(M2F_EINVAL, "%s: bad arguments", fn);
  const int OH = (H - 1) / 2 + 1, OW = (W - 1) / 2 + 1;
  const int64_t total = planes * OH * OW;
  if (total == 0) return m2f::ok();
  hipStream_t st = static_cast<hipStream_t>(stream);
  const unsigned grid = m2f::ceil_div(total, 256);
  if (dtype == M2F_BF16)
    maxpool3s2_fwd<__bf16><<<grid, 256, 0, st>>>(static_cast<const __bf16*>(x), static_cast<__bf16*>(y), window, H,
                                                 W, OH, OW, total);
  else if (dtype == M2F_F16)
    maxpool3s2_fwd<_Float16><<<grid, 256, 0, st>>>(static_cast<const _Float16*>(x), static_cast<_Float16*>(y), window,
                                                   H, W, OH, OW, total);
  else if (dtype == M2F_F32)
    maxpool3s2_fwd<float><<<grid, 256, 0, st>>>(static_cast<const float*>(x), static_cast<float*>(y), window, H, W,
                                                OH, OW, total);
  else
    return m2f::fail(M2F_EUNSUPPORTED, "%s: dtype %d", fn, dtype);
  return m2f::check_launch(fn);
}

extern "C" int m2f_maxpool3s2_bwd(const void* grad_y, const uint8_t* window, void* grad_x, int64_t planes, int H,
                                  int W, int dtype, void* stream) {
  const char* fn = "m2f_maxpool3s2_bwd";
  if (!grad_y || !window || !grad_x || planes < 0 || H <= 0 || W <= 0)
    return m2f::fail(M2F_EINVAL, "%s: bad arguments", fn);
  const int OH = (H - 1) / 2 + 1, OW = (W - 1) / 2 + 1;
  const int64_t total = planes * H * W;
  if (total == 0) return m2f::ok();
  hipStream_t st = static_cast<hipStream_t>(stream);
  if (W % 8 == 0 && m2f::aligned(grad_x, 16) && (dtype == M2F_BF16 || dtype == M2F_F16 || dtype == M2F_F32)) {
    const int64_t total8 = total / 8;
    const unsigned g8 = m2f::ceil_div(total8, 256);
    if (dtype == M2F_BF16)
      maxpool3s2_bwd8<__bf16><<<g8, 256, 0, st>>>(static_cast<const __bf16*>(grad_y), window,
                                                   static_cast<__bf16*>(grad_x), H, W, OH, OW, total8);
    else if (dtype == M2F_F16)
      maxpool3s2_bwd8<_Float16><<<g8, 256, 0, st>>>(static_cast<const _Float16*>(grad_y), window,
                                                     static_cast<_Float16*>(grad_x), H, W, OH, OW, total8);
    else
      maxpool3s2_bwd8<float><<<g8, 256, 0, st>>>(static_cast<const float*>(grad_y), window,
                                                  static_cast<float*>(grad_x), H, W, OH, OW, total8);
    return m2f::check_launch(fn);
  }
  const unsigned grid = m2f::ceil_div(total, 256);
  if (dtype == M2F_BF16)
    maxpool3s2_bwd<__bf16><<<grid, 256, 0, st>>>(static_cast<const __bf16*>(grad_y), window,
                                                 static_cast<__bf16*>(grad_x), H, W, OH, OW, total);
  else if (dtype == M2F_F16)
    maxpool3s2_bwd<_Float16><<<grid, 256, 0, st>>>(static_cast<const _Float16*>(grad_y), window,
                                                   static_cast<_Float16*>(grad_x), H, W, OH, OW, total);
  else if (dtype == M2F_F32)
    maxpool3s2_bwd<float><<<grid, 256, 0, st>>>(static_cast<const float*>(grad_y), window,
                                                static_cast<float*>(grad_x), H, W, OH, OW, total);
  else
    return m2f::fail(M2F_EUNSUPPORTED, "%s: dtype %d", fn, dtype);
  return m2f::check_launch(fn);
}

// ---------------------------------------------------------------------------------------------------
// Batched fp32 transpose out[b][q][r] = in[b][r][q] through 64x64 LDS tiles (both sides coalesced): the
// pixel decoder's level flatten, cat([x_l.flatten(2).transpose(1, 2)], 1) (msdeformattn.py:64-74), and its
// backward, without the library's strided cat.
// ---------------------------------------------------------------------------------------------------
namespace {

__global__ void __launch_bounds__(256) transpose_f32(const float* __restrict__ in, int64_t in_bs, int64_t in_ld,
                                                    float* __restrict__ out, int64_t out_bs, int64_t out_ld, int R,
                                                    int Q) {
  __shared__ float tile[64][65];
  const int b = blockIdx.z;
  const int r0 = blockIdx.y * 64, q0 = blockIdx.x * 64;
  const int tx = threadIdx.x & 63, ty = threadIdx.x >> 6;
  const float* ip = in + b * in_bs;
  float* op = out + b * out_bs;
  // all 16 loads in flight before any is used: an out-of-range element loads element 0 (R, Q > 0) and fills a tile
  // entry no in-range output reads (a guarded load per element had been 16 dependent round trips)
  float v[16];
#pragma unroll
  for (int k = 0; k < 16; ++k) {
    const int r = r0 + ty + 4 * k, q = q0 + tx;
    v[k] = ip[(r < R && q < Q) ? static_cast<int64_t>(r) * in_ld + q : 0];
  }
#pragma unroll
  for (int k = 0; k < 16; ++k) tile[ty + 4 * k][tx] = v[k];
  __syncthreads();
#pragma unroll
  for (int k = 0; k < 16; ++k) v[k] = tile[tx][ty + 4 * k];
#pragma unroll
  for (int k = 0; k < 16; ++k) {
    const int q = q0 + ty + 4 * k, r = r0 + tx;
    if (r < R && q < Q) op[static_cast<int64_t>(q) * out_ld + r] = v[k];
  }
}

}  // namespace

extern "C" int m2f_transpose_f32(const float* in, int64_t in_bs, int64_t in_ld, float* out, int64_t out_bs,
                                 int64_t out_ld, int B, int R, int Q, void* stream) {
  const char* fn = "m2f_transpose_f32";
  if (!in || !out || B < 0 || R < 0 || Q < 0 || in_ld < Q || out_ld < R)
    return m2f::fail(M2F_EINVAL, "%s: bad arguments", fn);
  if (B == 0 || R == 0 || Q == 0) return m2f::ok();
  if (B > 65535) return m2f::fail(M2F_EUNSUPPORTED, "%s: batch %d > 65535", fn, B);
  const dim3 grid((Q + 63) / 64, (R + 63) / 64, B);
  transpose_f32<<<grid, 256, 0, static_cast<hipStream_t>(stream)>>>(in, in_bs, in_ld, out, out_bs, out_ld, R, Q);
  return m2f::check_launch(fn);
}

// ---------------------------------------------------------------------------------------------------
// Column sums in fp32 of a row-major (rows, cols) matrix: out[c] = sum_r src[r][c] -- the bias / broadcast-add
// gradients over the decoder's memory tokens and the level embeddings.  1024-row chunks write fp32 partials
// (16-byte row vectors, row lanes added in order through LDS), then a second kernel adds the chunks in order: the same result every call, and no memset (torch's reduction of a
// long column to few outputs zeroes cross-block semaphores with one, which the runtime's graph packet capture
// replays wrongly).
namespace {

constexpr int kColsumRows = 1024;   // rows per chunk (at most 512 chunks)

int64_t colsum_chunks(int64_t rows) {
  int64_t n = (rows + kColsumRows - 1) / kColsumRows;
  return std::max<int64_t>(1, std::min<int64_t>(n, 512));
}

template <typename T, int V>
__device__ __forceinline__ void load_cols(const T* p, float (&v)[V]) {
  if constexpr (V == 8 && sizeof(T) == 2) {
    const uint4 u = *reinterpret_cast<const uint4*>(p);
    const T* e = reinterpret_cast<const T*>(&u);
#pragma unroll
    for (int i = 0; i < 8; ++i) v[i] = static_cast<float>(e[i]);
  } else if constexpr (V == 8) {
    const float4 a = *reinterpret_cast<const float4*>(p), b = *reinterpret_cast<const float4*>(p + 4);
    v[0] = a.x; v[1] = a.y; v[2] = a.z; v[3] = a.w; v[4] = b.x; v[5] = b.y; v[6] = b.z; v[7] = b.w;
  } else {
#pragma unroll
    for (int i = 0; i < V; ++i) v[i] = static_cast<float>(p[i]);
  }
}

// block: 64 columns x one chunk of rows; thread: V consecutive columns (V = 8: one 16- or 32-byte vector per row,
// rows 16-byte aligned) of every (256 V / 64)-th row, then the row lanes are added in order through LDS
template <typename T, int V>
__global__ void __launch_bounds__(256) colsum_part_kernel(const T* __restrict__ src, int64_t rows, int cols,
                                                          int64_t rows_per, float* __restrict__ part) {
  constexpr int TPR = 64 / V, RL = 256 / TPR;   // threads per row, row lanes
  __shared__ float red[RL][65];
  const int cg = threadIdx.x % TPR, rl = threadIdx.x / TPR;
  const int c0 = blockIdx.x * 64 + cg * V;
  const int64_t r0 = blockIdx.y * rows_per, r1 = std::min<int64_t>(rows, r0 + rows_per);
  float acc[V];
#pragma unroll
  for (int i = 0; i < V; ++i) acc[i] = 0.f;
  if (c0 < cols) {
    const T* p = src + c0;
#pragma unroll 4
    for (int64_t r = r0 + rl; r < r1; r += RL) {
      float v[V];
      load_cols<T, V>(p + r * cols, v);
#pragma unroll
      for (int i = 0; i < V; ++i) acc[i] += v[i];
    }
  }
#pragma unroll
  for (int i = 0; i < V; ++i) red[rl][cg * V + i] = acc[i];
  __syncthreads();
  if (threadIdx.x < 64) {
    const int c = blockIdx.x * 64 + threadIdx.x;
    float s = 0.f;
    for (int k = 0; k < RL; ++k) s += red[k][threadIdx.x];
    if (c < cols) part[blockIdx.y * static_cast<int64_t>(cols) + c] = s;
  }
}

// block: 64 columns; wave w adds chunks w, w + 4, ..., then the four waves in order
__global__ void __launch_bounds__(256) colsum_final_kernel(const float* __restrict__ part, int chunks, int cols,
                                                           float* __restrict__ out) {
  __shared__ float red[4][64];
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int c = blockIdx.x * 64 + lane;
  float s = 0.f;
  if (c < cols)
    for (int k = w; k < chunks; k += 4) s += part[static_cast<int64_t>(k) * cols + c];
  red[w][lane] = s;
  __syncthreads();
  if (w == 0 && c < cols) out[c] = ((red[0][lane] + red[1][lane]) + red[2][lane]) + red[3][lane];
}

}  // namespace

extern "C" int m2f_colsum_workspace(int64_t rows, int cols, int64_t* workspace_floats) {
  if (rows < 0 || cols <= 0 || !workspace_floats) return m2f::fail(M2F_EINVAL, "m2f_colsum_workspace: bad arguments");
  *workspace_floats = colsum_chunks(rows) * cols;
  return m2f::ok();
}

extern "C" int m2f_colsum(int dtype, const void* src, int64_t rows, int cols, float* workspace,
                          int64_t workspace_floats, float* out, void* stream) {
  const char* fn = "m2f_colsum";
  if (!src || !workspace || !out || rows < 0 || cols <= 0) return m2f::fail(M2F_EINVAL, "%s: bad arguments", fn);
  const int64_t chunks = colsum_chunks(rows);
  if (workspace_floats < chunks * cols)
    return m2f::fail(M2F_EINVAL, "%s: workspace %lld < %lld floats", fn, static_cast<long long>(workspace_floats),
                     static_cast<long long>(chunks * cols));
  if (cols > 65535 * 64) return m2f::fail(M2F_EUNSUPPORTED, "%s: %d columns", fn, cols);
  hipStream_t st = static_cast<hipStream_t>(stream);
  const int64_t rows_per = std::max<int64_t>(1, (rows + chunks - 1) / chunks);
  const dim3 grid((cols + 63) / 64, static_cast<unsigned>(chunks));
  // 8-column vectors when every row starts 16-byte aligned and cols % 8 == 0, else one column per thread
  const int esz = dtype == M2F_F32 ? 4 : 2;
  const bool vec = cols % 8 == 0 && m2f::aligned(src, 16) && (static_cast<int64_t>(cols) * esz) % 16 == 0;
#define M2F_COLSUM(T)                                                                                                   \
  (vec ? colsum_part_kernel<T, 8><<<grid, 256, 0, st>>>(static_cast<const T*>(src), rows, cols, rows_per, workspace)   \
       : colsum_part_kernel<T, 1><<<grid, 256, 0, st>>>(static_cast<const T*>(src), rows, cols, rows_per, workspace))
  switch (dtype) {
    case M2F_F32: M2F_COLSUM(float); break;
    case M2F_F16: M2F_COLSUM(_Float16); break;
    case M2F_BF16: M2F_COLSUM(__bf16); break;
    default: return m2f::fail(M2F_EUNSUPPORTED, "%s: dtype %d", fn, dtype);
  }
#undef M2F_COLSUM
  colsum_final_kernel<<<(cols + 63) / 64, 256, 0, st>>>(workspace, static_cast<int>(chunks), cols, out);
  return m2f::check_launch(fn);
}

// ---------------------------------------------------------------------------------------------------
// Achievable-HBM probe ("measure achievable peaks with a stream kernel"): out = in over
// n16 16-byte vectors.  mode 0: one pass, each thread copies 4 vectors a block-width apart (plain loads and
// stores, ~n16 / 1024 workgroups); mode 1: a fixed grid of 8 workgroups per CU striding over the buffer with
// nontemporal loads and stores.  Bytes moved = 32 * n16.
// ---------------------------------------------------------------------------------------------------
namespace {

typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));

__global__ void __launch_bounds__(256) stream_copy_kernel(const u32x4* __restrict__ in, u32x4* __restrict__ out,
                                                         int64_t n16) {
  const int64_t i = blockIdx.x * 1024ll + threadIdx.x;
  if (i + 768 < n16) {
    const u32x4 a = in[i], b = in[i + 256], c = in[i + 512], d = in[i + 768];
    out[i] = a;
    out[i + 256] = b;
    out[i + 512] = c;
    out[i + 768] = d;
  } else {
    for (int64_t k = i; k < n16 && k < i + 1024; k += 256) out[k] = in[k];
  }
}

__global__ void __launch_bounds__(256) stream_copy_nt_kernel(const u32x4* __restrict__ in, u32x4* __restrict__ out,
                                                            int64_t n16) {
  const int64_t stride = static_cast<int64_t>(gridDim.x) * blockDim.x;
  int64_t i = blockIdx.x * static_cast<int64_t>(blockDim.x) + threadIdx.x;
  for (; i + 3 * stride < n16; i += 4 * stride) {  // four independent 16-byte loads in flight per lane
    const u32x4 a = __builtin_nontemporal_load(in + i);
    const u32x4 b = __builtin_nontemporal_load(in + i + stride);
    const u32x4 c = __builtin_nontemporal_load(in + i + 2 * stride);
    const u32x4 d = __builtin_nontemporal_load(in + i + 3 * stride);
    __builtin_nontemporal_store(a, out + i);
    __builtin_nontemporal_store(b, out + i + stride);
    __builtin_nontemporal_store(c, out + i + 2 * stride);
    __builtin_nontemporal_store(d, out + i + 3 * stride);
  }
  for (; i < n16; i += stride) __builtin_nontemporal_store(__builtin_nontemporal_load(in + i), out + i);
}

}  // namespace

extern "C" int m2f_stream_copy(const void* in, void* out, int64_t nbytes, int mode, void* stream) {
  const char* fn = "m2f_stream_copy";
  if (!in || !out || nbytes < 0 || mode < 0 || mode > 1) return m2f::fail(M2F_EINVAL, "%s: bad arguments", fn);
  if (nbytes % 16 || !m2f::aligned(in, 16) || !m2f::aligned(out, 16))
    return m2f::fail(M2F_EUNSUPPORTED, "%s: needs 16-byte aligned buffers and nbytes %% 16 == 0", fn);
  const int64_t n16 = nbytes / 16;
  if (n16 == 0) return m2f::ok();
  hipStream_t st = static_cast<hipStream_t>(stream);
  const u32x4* src = static_cast<const u32x4*>(in);
  u32x4* dst = static_cast<u32x4*>(out);
  if (mode == 0) {
    const int64_t blocks = (n16 + 1023) / 1024;
    if (blocks > 0x7fffffff) return m2f::fail(M2F_EUNSUPPORTED, "%s: too large", fn);
    stream_copy_kernel<<<static_cast<unsigned>(blocks), 256, 0, st>>>(src, dst, n16);
  } else {
    const unsigned grid = static_cast<unsigned>(std::min<int64_t>(2048, m2f::ceil_div(n16, 256)));
    stream_copy_nt_kernel<<<grid, 256, 0, st>>>(src, dst, n16);
  }
  return m2f::check_launch(fn);
}

// ---------------------------------------------------------------------------------------------------
// Achievable-gather probe: the MSDA kernels' binding path is the L2-resident gather of 128-byte value rows
// (one head's rows of one image, 2.75 MB at 1024^2, stay in an XCD's 4 MB L2), not HBM.  An 8-lane group
// reads one pseudo-random 128-byte row of `table` (rows x 32 floats) per step, as the MSDA kernels' groups
// read a sample's corner rows (a float4 per lane), four rows in flight per lane; n rows in total.  Row ids are
// hashed from the step index (no index traffic).  Gathered bytes = 128 * n; out gets one float per lane.
// ---------------------------------------------------------------------------------------------------
namespace {

__device__ __forceinline__ uint32_t probe_hash(uint64_t x) {
  x ^= x >> 33;
  x *= 0xff51afd7ed558ccdull;
  x ^= x >> 33;
  return static_cast<uint32_t>(x);
}

__global__ void __launch_bounds__(256) gather_probe_kernel(const float4* __restrict__ table, uint32_t rows,
                                                          int64_t n, float* __restrict__ out) {
  const int64_t gid = blockIdx.x * static_cast<int64_t>(blockDim.x) + threadIdx.x;
  const int64_t groups = static_cast<int64_t>(gridDim.x) * blockDim.x / 8;
  const int j = threadIdx.x & 7;
  float4 acc = make_float4(0.f, 0.f, 0.f, 0.f);
  int64_t i = gid >> 3;
  for (; i + 3 * groups < n; i += 4 * groups) {
    const float4 a = table[static_cast<int64_t>(probe_hash(i) % rows) * 8 + j];
    const float4 b = table[static_cast<int64_t>(probe_hash(i + groups) % rows) * 8 + j];
    const float4 c = table[static_cast<int64_t>(probe_hash(i + 2 * groups) % rows) * 8 + j];
    const float4 d = table[static_cast<int64_t>(probe_hash(i + 3 * groups) % rows) * 8 + j];
    acc.x += (a.x + b.x) + (c.x + d.x);
    acc.y += (a.y + b.y) + (c.y + d.y);
    acc.z += (a.z + b.z) + (c.z + d.z);
    acc.w += (a.w + b.w) + (c.w + d.w);
  }
  for (; i < n; i += groups) {
    const float4 a = table[static_cast<int64_t>(probe_hash(i) % rows) * 8 + j];
    acc.x += a.x; acc.y += a.y; acc.z += a.z; acc.w += a.w;
  }
  out[gid] = (acc.x + acc.y) + (acc.z + acc.w);
}

}  // namespace

extern "C" int m2f_gather_probe(const float* table, int rows, int64_t n, float* out, int out_len, void* stream) {
  const char* fn = "m2f_gather_probe";
  if (!table || !out || rows <= 0 || n < 0 || !m2f::aligned(table, 16)) return m2f::fail(M2F_EINVAL, "%s: bad arguments", fn);
  const int grid = 2048;   // 8 workgroups of 4 waves per CU
  if (out_len < grid * 256) return m2f::fail(M2F_EINVAL, "%s: out needs %d floats", fn, grid * 256);
  gather_probe_kernel<<<grid, 256, 0, static_cast<hipStream_t>(stream)>>>(reinterpret_cast<const float4*>(table),
                                                                          static_cast<uint32_t>(rows), n, out);
  return m2f::check_launch(fn);
}

// ------------------------------------------------------------------------------------------------
// m2f::zero_async: a grid-stride fill with 16-byte stores (byte stores for an unaligned head / tail)
// ------------------------------------------------------------------------------------------------
namespace {
__global__ void __launch_bounds__(256) zero16_kernel(uint4* __restrict__ p, size_t n16) {
  const uint4 z = {0u, 0u, 0u, 0u};
  for (size_t i = blockIdx.x * 256ull + threadIdx.x; i < n16; i += static_cast<size_t>(gridDim.x) * 256) p[i] = z;
}
__global__ void __launch_bounds__(256) zero1_kernel(unsigned char* __restrict__ p, size_t n) {
  for (size_t i = blockIdx.x * 256ull + threadIdx.x; i < n; i += static_cast<size_t>(gridDim.x) * 256) p[i] = 0;
}
// rows x cols floats at row stride ld (floats): one grid-stride pass over the rows x cols elements
__global__ void __launch_bounds__(256) zero2d_f32_kernel(float* __restrict__ p, int64_t ld, int64_t cols, int64_t n) {
  for (int64_t i = blockIdx.x * 256ll + threadIdx.x; i < n; i += static_cast<int64_t>(gridDim.x) * 256) {
    const int64_t r = i / cols;
    p[r * ld + (i - r * cols)] = 0.f;
  }
}
}  // namespace

namespace m2f {
hipError_t zero_async(void* p, size_t bytes, hipStream_t st) {
  if (bytes == 0) return hipSuccess;
  unsigned char* b = static_cast<unsigned char*>(p);
  const size_t head = std::min(bytes, (16 - (reinterpret_cast<uintptr_t>(b) & 15)) & 15);
  const size_t n16 = (bytes - head) / 16, tail = bytes - head - n16 * 16;
  if (head) zero1_kernel<<<1, 256, 0, st>>>(b, head);
  if (n16) {
    const size_t blocks = std::min<size_t>((n16 + 255) / 256, 4096);
    zero16_kernel<<<static_cast<unsigned>(blocks), 256, 0, st>>>(reinterpret_cast<uint4*>(b + head), n16);
  }
  if (tail) zero1_kernel<<<1, 256, 0, st>>>(b + head + n16 * 16, tail);
  return hipGetLastError();
}

hipError_t zero2d_f32_async(float* p, int64_t ld, int64_t cols, int64_t rows, hipStream_t st) {
  if (rows <= 0 || cols <= 0) return hipSuccess;
  if (ld == cols) return zero_async(p, static_cast<size_t>(rows * cols) * sizeof(float), st);
  const int64_t n = rows * cols;
  const int64_t blocks = std::min<int64_t>((n + 255) / 256, 4096);
  zero2d_f32_kernel<<<static_cast<unsigned>(blocks), 256, 0, st>>>(p, ld, cols, n);
  return hipGetLastError();
}

int set_max_lds(const void* kernel, int bytes, const char* fn) {
  // one hipFuncSetAttribute per (kernel, device, limit), thread-safe; the attribute is per device, so a process that
  // launches on several devices sets it on each
  static std::mutex mu;
  static std::set<std::tuple<const void*, int, int>> done;
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess) return fail(M2F_ELAUNCH, "%s: hipGetDevice failed", fn);
  std::lock_guard<std::mutex> lock(mu);
  const auto key = std::make_tuple(kernel, dev, bytes);
  if (done.count(key)) return M2F_OK;
  const hipError_t e = hipFuncSetAttribute(kernel, hipFuncAttributeMaxDynamicSharedMemorySize, bytes);
  if (e != hipSuccess)
    return fail(M2F_ELAUNCH, "%s: hipFuncSetAttribute(MaxDynamicSharedMemorySize = %d) on device %d: %s", fn, bytes, dev,
                hipGetErrorString(e));
  done.insert(key);
  return M2F_OK;
}
}  // namespace m2f
