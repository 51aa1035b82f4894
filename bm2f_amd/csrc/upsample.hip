// FPN merge of the pixel decoder (msdeformattn.py:343-349):
//     y = lateral + F.interpolate(coarse, size=lateral.shape[-2:], mode="bilinear", align_corners=False)
// for the exact 2x case (stride 8 -> stride 4), fp32, NCHW output, as one pass: the library runs the
// upsample (NHWC, because the encoder's map arrives as a transposed (N, HW, C) view) and then a mixed-layout
// add that cannot vectorise (2.9 ms fwd + 1.2 ms bwd at bs16 256x256x256, tools/fpn_bench.py).
//
// Forward: a thread owns 4 consecutive output pixels of one (n, c) row; the four source taps follow
// upsample_bilinear2d's align_corners=False rule literally (src = 0.5 (dst + 0.5) - 0.5 clamped at 0,
// i1 = i0 + (i0 < in - 1), same lambda products and order), then the lateral is added.  The C ABI takes
// the coarse map through arbitrary strides; the Python layer (conv_ops.Upsample2xAdd) nevertheless makes it
// contiguous first, because a strided read of the transposed (N, HW, C) view costs a cache line per lane
// and tap (2.6 ms vs 1.0 ms including the copy at bs16 128->256), so from Python the kernel always sees
// unit-stride rows; the strided form is exercised through the C ABI by tests/test_conv_gpu.py.
// Backward: grad_lateral is grad_out itself; grad_coarse is a gather (no atomics, deterministic): each
// source pixel sums the <= 4 x 4 output pixels whose taps touch it, with the forward's weights.
#include "bm2f.h"
#include "common.h"

#include <hip/hip_runtime.h>

namespace {

using f4 = __attribute__((__vector_size__(4 * sizeof(float)))) float;

struct Tap {
  int i0, i1;
  float l0, l1;
};

// upsample_bilinear2d source index for output o (scale in/out = 0.5, align_corners=False)
__device__ __forceinline__ Tap tap2x(int o, int in) {
  float src = 0.5f * (static_cast<float>(o) + 0.5f) - 0.5f;
  src = src < 0.f ? 0.f : src;
  Tap t;
  t.i0 = static_cast<int>(src);
  t.i1 = t.i0 + (t.i0 < in - 1 ? 1 : 0);
  t.l1 = src - static_cast<float>(t.i0);
  t.l0 = 1.f - t.l1;
  return t;
}

// weight of source index i in output o's interpolation (both taps may be i at the last index)
__device__ __forceinline__ float wgt2x(int o, int i, int in) {
  const Tap t = tap2x(o, in);
  return (t.i0 == i ? t.l0 : 0.f) + (t.i1 == i ? t.l1 : 0.f);
}

__global__ void __launch_bounds__(256) up2x_add_fwd(const float* __restrict__ src, int64_t sN, int64_t sC,
                                                    int64_t sY, int64_t sX, const float* __restrict__ lat,
                                                    float* __restrict__ out, int C, int h, int w, int64_t nvec) {
  const int64_t t = blockIdx.x * static_cast<int64_t>(blockDim.x) + threadIdx.x;
  if (t >= nvec) return;
  const int W2 = 2 * w, H2 = 2 * h, qv = W2 / 4;
  const int ox0 = static_cast<int>(t % qv) * 4;
  const int64_t r = t / qv;  // (n, c, oy)
  const int oy = static_cast<int>(r % H2);
  const int64_t nc = r / H2;
  const int c = static_cast<int>(nc % C);
  const int64_t n = nc / C;
  const float* base = src + n * sN + c * sC;
  const Tap ty = tap2x(oy, h);
  const float* r0 = base + ty.i0 * sY;
  const float* r1 = base + ty.i1 * sY;
  const int64_t o = r * W2 + ox0;
  f4 v = *reinterpret_cast<const f4*>(lat + o);
#pragma unroll
  for (int e = 0; e < 4; ++e) {
    const Tap tx = tap2x(ox0 + e, w);
    const float val = ty.l0 * (tx.l0 * r0[tx.i0 * sX] + tx.l1 * r0[tx.i1 * sX]) +
                      ty.l1 * (tx.l0 * r1[tx.i0 * sX] + tx.l1 * r1[tx.i1 * sX]);
    v[e] = v[e] + val;
  }
  *reinterpret_cast<f4*>(out + o) = v;
}

// contiguous source rows (sX == 1): the four output pixels of a thread read source columns 2t-1 .. 2t+2
// (clamped) only, so each row is loaded once into a 4-value window (8 loads instead of 16); same taps,
// same products and order as up2x_add_fwd (FMA contraction may differ: equal to fp32 rounding)
__device__ __forceinline__ float pick4(const float (&v)[4], int j) {
  return j == 0 ? v[0] : (j == 1 ? v[1] : (j == 2 ? v[2] : v[3]));
}

__global__ void __launch_bounds__(256) up2x_add_fwd_rows(const float* __restrict__ src, int64_t sN, int64_t sC,
                                                         int64_t sY, const float* __restrict__ lat,
                                                         float* __restrict__ out, int C, int h, int w, int64_t nvec) {
  const int64_t t = blockIdx.x * static_cast<int64_t>(blockDim.x) + threadIdx.x;
  if (t >= nvec) return;
  const int W2 = 2 * w, H2 = 2 * h, qv = W2 / 4;
  const int q = static_cast<int>(t % qv), ox0 = q * 4, cb = 2 * q - 1;
  const int64_t r = t / qv;
  const int oy = static_cast<int>(r % H2);
  const int64_t nc = r / H2;
  const int c = static_cast<int>(nc % C);
  const int64_t n = nc / C;
  const float* base = src + n * sN + c * sC;
  const Tap ty = tap2x(oy, h);
  const float* r0 = base + ty.i0 * sY;
  const float* r1 = base + ty.i1 * sY;
  float v0[4], v1[4];
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const int col = min(max(cb + j, 0), w - 1);
    v0[j] = r0[col];
    v1[j] = r1[col];
  }
  const int64_t o = r * W2 + ox0;
  f4 v = *reinterpret_cast<const f4*>(lat + o);
#pragma unroll
  for (int e = 0; e < 4; ++e) {
    const Tap tx = tap2x(ox0 + e, w);
    const int j0 = tx.i0 - cb, j1 = tx.i1 - cb;
    const float val = ty.l0 * (tx.l0 * pick4(v0, j0) + tx.l1 * pick4(v0, j1)) +
                      ty.l1 * (tx.l0 * pick4(v1, j0) + tx.l1 * pick4(v1, j1));
    v[e] = v[e] + val;
  }
  *reinterpret_cast<f4*>(out + o) = v;
}

// grad_src[n][c][y][x] (contiguous) = sum over oy in [2y-1, 2y+2], ox in [2x-1, 2x+2] of
// wy(oy, y) wx(ox, x) g[n][c][oy][ox]
__global__ void __launch_bounds__(256) up2x_bwd(const float* __restrict__ g, float* __restrict__ gsrc, int h, int w,
                                                int64_t n_in) {
  const int64_t t = blockIdx.x * static_cast<int64_t>(blockDim.x) + threadIdx.x;
  if (t >= n_in) return;
  const int x = static_cast<int>(t % w);
  const int64_t r = t / w;
  const int y = static_cast<int>(r % h);
  const int64_t plane = r / h;
  const int H2 = 2 * h, W2 = 2 * w;
  const float* gp = g + plane * H2 * W2;
  float acc = 0.f;
#pragma unroll
  for (int dy = -1; dy <= 2; ++dy) {
    const int oy = 2 * y + dy;
    if (oy < 0 || oy >= H2) continue;
    const float wy = wgt2x(oy, y, h);
    if (wy == 0.f) continue;
    float row = 0.f;
#pragma unroll
    for (int dx = -1; dx <= 2; ++dx) {
      const int ox = 2 * x + dx;
      if (ox < 0 || ox >= W2) continue;
      row += wgt2x(ox, x, w) * gp[static_cast<int64_t>(oy) * W2 + ox];
    }
    acc += wy * row;
  }
  gsrc[t] = acc;
}

// two horizontally adjacent source pixels per thread (w even): each output row segment 4k-1 .. 4k+4 is one
// aligned float4 plus two edge values, shared by both pixels; same sums in the same order as up2x_bwd
__global__ void __launch_bounds__(256) up2x_bwd2(const float* __restrict__ g, float* __restrict__ gsrc, int h, int w,
                                                 int64_t n_pairs) {
  const int64_t t = blockIdx.x * static_cast<int64_t>(blockDim.x) + threadIdx.x;
  if (t >= n_pairs) return;
  const int wp = w / 2;
  const int k = static_cast<int>(t % wp), x0 = 2 * k;
  const int64_t r = t / wp;
  const int y = static_cast<int>(r % h);
  const int64_t plane = r / h;
  const int H2 = 2 * h, W2 = 2 * w;
  const float* gp = g + plane * H2 * W2;
  float wa[6], wb[6];   // column weights of cols 4k-1 .. 4k+4 for source pixels x0, x0+1
#pragma unroll
  for (int c = 0; c < 6; ++c) {
    const int ox = 4 * k - 1 + c;
    const bool ok = ox >= 0 && ox < W2;
    wa[c] = ok && c < 4 ? wgt2x(ox, x0, w) : 0.f;
    wb[c] = ok && c >= 2 ? wgt2x(ox, x0 + 1, w) : 0.f;
  }
  float acc_a = 0.f, acc_b = 0.f;
#pragma unroll
  for (int dy = -1; dy <= 2; ++dy) {
    const int oy = 2 * y + dy;
    if (oy < 0 || oy >= H2) continue;
    const float wy = wgt2x(oy, y, h);
    if (wy == 0.f) continue;
    const float* row = gp + static_cast<int64_t>(oy) * W2;
    const f4 mid = *reinterpret_cast<const f4*>(row + 4 * k);
    const float v[6] = {4 * k - 1 >= 0 ? row[4 * k - 1] : 0.f, mid[0], mid[1], mid[2], mid[3],
                        4 * k + 4 < W2 ? row[4 * k + 4] : 0.f};
    float ra = 0.f, rb = 0.f;
#pragma unroll
    for (int c = 0; c < 4; ++c) {   // up2x_bwd's dx order: cols 2x-1 .. 2x+2, skipping those outside
      const int oxa = 4 * k - 1 + c, oxb = 4 * k + 1 + c;
      if (oxa >= 0 && oxa < W2) ra += wa[c] * v[c];
      if (oxb >= 0 && oxb < W2) rb += wb[c + 2] * v[c + 2];
    }
    acc_a += wy * ra;
    acc_b += wy * rb;
  }
  float* dst = gsrc + (plane * h + y) * static_cast<int64_t>(w) + x0;
  dst[0] = acc_a;
  dst[1] = acc_b;
}

}  // namespace

extern "C" int m2f_upsample2x_add_fwd_f32(const float* src, int64_t sN, int64_t sC, int64_t sY, int64_t sX,
                                          const float* lateral, float* out, int N, int C, int h, int w,
                                          void* stream) {
  const char* fn = "m2f_upsample2x_add_fwd_f32";
  if (!src || !lateral || !out) return m2f::fail(M2F_EINVAL, "%s: null pointer", fn);
  if (N < 0 || C <= 0 || h <= 0 || w <= 0) return m2f::fail(M2F_EINVAL, "%s: bad sizes", fn);
  if ((2 * w) % 4 || !m2f::aligned(lateral, 16) || !m2f::aligned(out, 16))
    return m2f::fail(M2F_EUNSUPPORTED, "%s: needs 2*w %% 4 == 0 and 16-byte aligned lateral/out", fn);
  const int64_t nvec = static_cast<int64_t>(N) * C * (2 * h) * (2 * w) / 4;
  if (nvec == 0) return m2f::ok();
  if (sX == 1)
    up2x_add_fwd_rows<<<m2f::ceil_div(nvec, 256), 256, 0, static_cast<hipStream_t>(stream)>>>(src, sN, sC, sY, lateral,
                                                                                            out, C, h, w, nvec);
  else
    up2x_add_fwd<<<m2f::ceil_div(nvec, 256), 256, 0, static_cast<hipStream_t>(stream)>>>(src, sN, sC, sY, sX, lateral,
                                                                                         out, C, h, w, nvec);
  return m2f::check_launch(fn);
}

extern "C" int m2f_upsample2x_bwd_f32(const float* grad_out, float* grad_src, int N, int C, int h, int w,
                                      void* stream) {
  const char* fn = "m2f_upsample2x_bwd_f32";
  if (!grad_out || !grad_src) return m2f::fail(M2F_EINVAL, "%s: null pointer", fn);
  if (N < 0 || C <= 0 || h <= 0 || w <= 0) return m2f::fail(M2F_EINVAL, "%s: bad sizes", fn);
  const int64_t n_in = static_cast<int64_t>(N) * C * h * w;
  if (n_in == 0) return m2f::ok();
  if (w % 2 == 0 && m2f::aligned(grad_out, 16)) {
    up2x_bwd2<<<m2f::ceil_div(n_in / 2, 256), 256, 0, static_cast<hipStream_t>(stream)>>>(grad_out, grad_src, h, w,
                                                                                          n_in / 2);
    return m2f::check_launch(fn);
  }
  up2x_bwd<<<m2f::ceil_div(n_in, 256), 256, 0, static_cast<hipStream_t>(stream)>>>(grad_out, grad_src, h, w, n_in);
  return m2f::check_launch(fn);
}
