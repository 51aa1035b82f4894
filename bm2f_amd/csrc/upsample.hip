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

// ---- channels-last source (the encoder's (N, HW, C) map seen as (N, C, h, w)): both directions LDS-tiled --------
// A block owns one output row oy (forward) / source row y (backward) of one image and kUpCT channels.  The channel
// axis is the unit-stride one of the (N, h, w, C) side and the x axis that of the NCHW side, so each side is read
// or written coalesced and the transpose happens in LDS (pitch kUpCT + 1 floats: the x-strided reads of one
// channel fall on distinct banks two apart).  Same taps, products and summation order as the NCHW kernels.
constexpr int kUpCT = 64;
constexpr int kUpPitch = kUpCT + 1;
constexpr int kUpMaxW = 256;   // LDS: forward 2 * w * kUpPitch floats, backward w * kUpPitch

__global__ void __launch_bounds__(256) up2x_add_fwd_nhwc(const float* __restrict__ src, int64_t sN,
                                                         const float* __restrict__ lat, float* __restrict__ out, int C,
                                                         int h, int w) {
  extern __shared__ float tile[];   // [2][w][kUpPitch]: source rows i0, i1 of this channel tile
  const int nct = C / kUpCT, H2 = 2 * h, W2 = 2 * w;
  const int ct = blockIdx.x % nct;
  const int r = blockIdx.x / nct;
  const int oy = r % H2, n = r / H2;
  const Tap ty = tap2x(oy, h);
  const int c4n = kUpCT / 4;
  for (int idx = threadIdx.x; idx < 2 * w * c4n; idx += blockDim.x) {
    const int sel = idx / (w * c4n), rem = idx - sel * w * c4n;
    const int x = rem / c4n, c4 = rem - x * c4n;
    const int iy = sel ? ty.i1 : ty.i0;
    const f4 v = *reinterpret_cast<const f4*>(src + n * sN + (static_cast<int64_t>(iy) * w + x) * C + ct * kUpCT + 4 * c4);
    float* d = tile + (sel * w + x) * kUpPitch + 4 * c4;
    d[0] = v[0]; d[1] = v[1]; d[2] = v[2]; d[3] = v[3];
  }
  __syncthreads();
  const int qv = W2 / 4;
  for (int it = threadIdx.x; it < kUpCT * qv; it += blockDim.x) {
    const int c = it / qv, q = it - c * qv, ox0 = 4 * q;
    const int64_t o = ((static_cast<int64_t>(n) * C + ct * kUpCT + c) * H2 + oy) * W2 + ox0;
    f4 v = *reinterpret_cast<const f4*>(lat + o);
    const float* r0 = tile + c;
    const float* r1 = tile + w * kUpPitch + c;
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      const Tap tx = tap2x(ox0 + e, w);
      const float val = ty.l0 * (tx.l0 * r0[tx.i0 * kUpPitch] + tx.l1 * r0[tx.i1 * kUpPitch]) +
                        ty.l1 * (tx.l0 * r1[tx.i0 * kUpPitch] + tx.l1 * r1[tx.i1 * kUpPitch]);
      v[e] = v[e] + val;
    }
    *reinterpret_cast<f4*>(out + o) = v;
  }
}

// grad_src (N, h, w, C) from grad_out (N, C, 2h, 2w): up2x_bwd2's sums per (channel, source pixel pair), staged
// in LDS and stored channel-contiguous
__global__ void __launch_bounds__(256) up2x_bwd_nhwc(const float* __restrict__ g, float* __restrict__ gsrc, int C,
                                                     int h, int w) {
  extern __shared__ float tile[];   // [w][kUpPitch]
  const int nct = C / kUpCT, H2 = 2 * h, W2 = 2 * w, wp = w / 2;
  const int ct = blockIdx.x % nct;
  const int r = blockIdx.x / nct;
  const int y = r % h, n = r / h;
  for (int it = threadIdx.x; it < kUpCT * wp; it += blockDim.x) {
    const int c = it / wp, k = it - c * wp, x0 = 2 * k;
    const float* gp = g + (static_cast<int64_t>(n) * C + ct * kUpCT + c) * H2 * W2;
    float wa[6], wb[6];
#pragma unroll
    for (int cc = 0; cc < 6; ++cc) {
      const int ox = 4 * k - 1 + cc;
      const bool ok = ox >= 0 && ox < W2;
      wa[cc] = ok && cc < 4 ? wgt2x(ox, x0, w) : 0.f;
      wb[cc] = ok && cc >= 2 ? wgt2x(ox, x0 + 1, w) : 0.f;
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
      for (int cc = 0; cc < 4; ++cc) {
        const int oxa = 4 * k - 1 + cc, oxb = 4 * k + 1 + cc;
        if (oxa >= 0 && oxa < W2) ra += wa[cc] * v[cc];
        if (oxb >= 0 && oxb < W2) rb += wb[cc + 2] * v[cc + 2];
      }
      acc_a += wy * ra;
      acc_b += wy * rb;
    }
    tile[x0 * kUpPitch + c] = acc_a;
    tile[(x0 + 1) * kUpPitch + c] = acc_b;
  }
  __syncthreads();
  const int c4n = kUpCT / 4;
  for (int idx = threadIdx.x; idx < w * c4n; idx += blockDim.x) {
    const int x = idx / c4n, c4 = idx - x * c4n;
    const float* s = tile + x * kUpPitch + 4 * c4;
    *reinterpret_cast<f4*>(gsrc + ((static_cast<int64_t>(n) * h + y) * w + x) * C + ct * kUpCT + 4 * c4) =
        f4{s[0], s[1], s[2], s[3]};
  }
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

// channels-last coarse map: src (N, h, w, C) with batch stride sN elements (>= h*w*C; the encoder's (N, S, C) output
// holds the level as a slice), lateral / out NCHW
extern "C" int m2f_upsample2x_add_fwd_nhwc_f32(const float* src, int64_t sN, const float* lateral, float* out, int N,
                                               int C, int h, int w, void* stream) {
  const char* fn = "m2f_upsample2x_add_fwd_nhwc_f32";
  if (!src || !lateral || !out) return m2f::fail(M2F_EINVAL, "%s: null pointer", fn);
  if (N < 0 || C <= 0 || h <= 0 || w <= 0) return m2f::fail(M2F_EINVAL, "%s: bad sizes", fn);
  // the output rows are stored as float4s of 2w columns: w must be even (an odd w would leave the last two
  // columns of every row unwritten and misalign the odd rows' vector accesses)
  if (C % kUpCT || w % 2 || w > kUpMaxW || sN % 4 || sN < static_cast<int64_t>(h) * w * C || !m2f::aligned(src, 16) ||
      !m2f::aligned(lateral, 16) || !m2f::aligned(out, 16))
    return m2f::fail(M2F_EUNSUPPORTED, "%s: needs C %% %d == 0, even w <= %d, sN %% 4 == 0, sN >= h*w*C and 16-byte "
                     "aligned buffers", fn, kUpCT, kUpMaxW);
  const int64_t nblk = static_cast<int64_t>(N) * 2 * h * (C / kUpCT);
  if (nblk == 0) return m2f::ok();
  if (nblk > 0x7fffffff) return m2f::fail(M2F_EUNSUPPORTED, "%s: too many blocks", fn);
  const size_t lds = static_cast<size_t>(2) * w * kUpPitch * sizeof(float);
  up2x_add_fwd_nhwc<<<static_cast<unsigned>(nblk), 256, lds, static_cast<hipStream_t>(stream)>>>(src, sN, lateral, out,
                                                                                                 C, h, w);
  return m2f::check_launch(fn);
}

// grad of the coarse map in channels-last layout: grad_src (N, h, w, C) contiguous from grad_out (N, C, 2h, 2w)
extern "C" int m2f_upsample2x_bwd_nhwc_f32(const float* grad_out, float* grad_src, int N, int C, int h, int w,
                                           void* stream) {
  const char* fn = "m2f_upsample2x_bwd_nhwc_f32";
  if (!grad_out || !grad_src) return m2f::fail(M2F_EINVAL, "%s: null pointer", fn);
  if (N < 0 || C <= 0 || h <= 0 || w <= 0) return m2f::fail(M2F_EINVAL, "%s: bad sizes", fn);
  if (C % kUpCT || w % 2 || w > kUpMaxW || !m2f::aligned(grad_out, 16) || !m2f::aligned(grad_src, 16))
    return m2f::fail(M2F_EUNSUPPORTED, "%s: needs C %% %d == 0, even w <= %d and 16-byte aligned buffers", fn, kUpCT,
                     kUpMaxW);
  const int64_t nblk = static_cast<int64_t>(N) * h * (C / kUpCT);
  if (nblk == 0) return m2f::ok();
  if (nblk > 0x7fffffff) return m2f::fail(M2F_EUNSUPPORTED, "%s: too many blocks", fn);
  const size_t lds = static_cast<size_t>(w) * kUpPitch * sizeof(float);
  up2x_bwd_nhwc<<<static_cast<unsigned>(nblk), 256, lds, static_cast<hipStream_t>(stream)>>>(grad_out, grad_src, C, h,
                                                                                             w);
  return m2f::check_launch(fn);
}
