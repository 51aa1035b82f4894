// Weak-supervision (box-supervised) target preparation, pairwise matching cost and pairwise loss.
//
// Reference (mask2former, SUP_TYPE "mask_projection_and_pairwise"):
//   target prep   maskformer_model.py:399-440  avg_pool 4x4 of the padded uint8 image, .byte(), skimage
//                 rgb2lab, weaksup_utils.py:34-57 colour similarity exp(-|lab_p - lab_q| / 2) over the 8
//                 dilated neighbours (unfold_wo_center, weaksup_utils.py:7-31), times the neighbour's
//                 image-mask value;
//   matcher cost  matcher.py:48-83 calculate_similarity_cost: s(p,q) = -log(sig(x_p)sig(x_q) +
//                 sig(-x_p)sig(-x_q)) in log space, weighted by (sim >= thr) * box, normalised per target;
//   loss          criterion.py:156-181 + 257-323: the same s on the matched masks, sum(s*T)/sum(T)/num_masks.
//
// The reference materialises (rows, 8, H, W) log-probability unfolds for each of them.  Here a workgroup
// owns a 16x64 pixel tile of one mask row, stages x and logsigmoid(x) of the tile plus its dilation halo
// in LDS, and evaluates the 8 neighbour terms per pixel in registers with one softplus each (hardware
// exp/log); the thresholded similarity is read as one byte of neighbour bits per pixel (bit k = sim[k] >=
// thr).  Out-of-image neighbours contribute 0, as F.unfold's zero padding of the log-probabilities makes
// them in the reference.  Sums are per-tile partials (deterministic; reduced by the caller).
#include "bm2f.h"
#include "common.h"

#include <hip/hip_runtime.h>

#include <cmath>

namespace {

constexpr int TH = 16, TW = 64, NT = 256;  // tile rows, cols, threads
constexpr int PPT = TH * TW / NT;           // pixels per thread: PPT consecutive rows of one column
constexpr int kMaxDil = 4;
constexpr int LW = TW + 2 * kMaxDil;  // LDS row pitch (fixed so the halo of any dilation <= 4 fits)
constexpr int LH = TH + 2 * kMaxDil;

// unfold_wo_center order: 3x3 taps row-major minus the centre; tap 7-k is the mirror of tap k
__device__ __forceinline__ int tap_dy(int k) { return (k < 3) ? -1 : (k < 5 ? 0 : 1); }
__device__ __forceinline__ int tap_dx(int k) {
  const int t = k < 4 ? k : k + 1;  // 3x3 index without the centre
  return t % 3 - 1;
}

constexpr float kLog2e = 1.4426950408889634f, kLn2 = 0.6931471805599453f;

// log(1 + exp(t)) for t <= 0 on the raw hardware exp2/log2 (one v_exp_f32 + one v_log_f32; 1 + e lies in
// [1, 2], so no denormal range fix-ups are needed)
__device__ __forceinline__ float softplus_neg(float t) {
  return kLn2 * __builtin_amdgcn_logf(1.f + __builtin_amdgcn_exp2f(t * kLog2e));
}

__device__ __forceinline__ float log_sigmoid(float x) {  // F.logsigmoid: min(x,0) - log1p(exp(-|x|))
  return fminf(x, 0.f) - softplus_neg(-fabsf(x));
}

// s(a,b) = -log(sig(a)sig(b) + sig(-a)sig(-b)) = -(logsig(a) + logsig(b) + softplus(-(a+b))): the
// reference's log-space form (criterion.py:175-179, with logsig(-x) = logsig(x) - x) reduced to one
// softplus per pair.  Pairs reaching outside the image are 0, as F.unfold's zero log-prob padding gives.
__device__ __forceinline__ float pair_term(float a, float fa, float b, float fb) {
  const float z = a + b;
  return -(fa + fb + fmaxf(-z, 0.f) + softplus_neg(-fabsf(z)));
}

__device__ __forceinline__ float sigmoid_neg(float t) {  // sig(-t), accurate in both tails
  const float e = __builtin_amdgcn_exp2f(-fabsf(t) * kLog2e);
  const float r = __builtin_amdgcn_rcpf(1.f + e);
  return t >= 0.f ? e * r : r;
}

// d s(a, b) / d a = sig(-(a+b)) - sig(-a)
__device__ __forceinline__ float pair_grad(float a, float sna, float b) { return sigmoid_neg(a + b) - sna; }

struct Tile {
  int ty0, tx0;
};

__device__ __forceinline__ Tile tile_of(int W) {
  const int ntx = (W + TW - 1) / TW;
  return {static_cast<int>(blockIdx.x / ntx) * TH, static_cast<int>(blockIdx.x % ntx) * TW};
}

// stage x and logsigmoid(x) of the tile + halo (values outside the image are never read)
__device__ __forceinline__ void stage_logits(const float* __restrict__ xr, int H, int W, int d, Tile t, float* lx,
                                             float* lf) {
  const int hh = TH + 2 * d;
  for (int i = threadIdx.x; i < hh * LW; i += NT) {
    const int yy = i / LW, xx = i % LW;  // LW is a constant: multiply-shift, no division
    const int gy = t.ty0 - d + yy, gx = t.tx0 - d + xx;
    float v = 0.f;
    if (xx < TW + 2 * d && gy >= 0 && gy < H && gx >= 0 && gx < W) v = xr[static_cast<int64_t>(gy) * W + gx];
    lx[i] = v;
    lf[i] = log_sigmoid(v);
  }
}

__device__ __forceinline__ bool inside(int y, int x, int H, int W) { return y >= 0 && y < H && x >= 0 && x < W; }

// bit k set when neighbour k of (y, x) lies in the image
__device__ __forceinline__ unsigned neighbours_inside(int y, int x, int H, int W, int d) {
  unsigned m = 0;
#pragma unroll
  for (int k = 0; k < 8; ++k) m |= (inside(y + tap_dy(k) * d, x + tap_dx(k) * d, H, W) ? 1u : 0u) << k;
  return m;
}

__device__ __forceinline__ float wave_sum(float v) {
  for (int off = 32; off > 0; off >>= 1) v += __shfl_xor(v, off);
  return v;
}

// MODE 0: out[r, p] = sum_k bit_k(p) s_k(p)                          (image-shared similarity map)
// MODE 1: part_num[r, tile] = sum_p w(p) sum_k bit_k s_k; part_den = sum_p w(p) popcount(bits(p))   (loss)
// MODE 2: out[r, k, p] = s_k(p)                                      (matcher, per-target similarity)
template <int MODE>
__global__ void __launch_bounds__(NT) pairwise_rows_kernel(const float* __restrict__ x, const int* __restrict__ x_row,
                                                           int H, int W, int d, const uint8_t* __restrict__ bits,
                                                           const int* __restrict__ t_row, const float* __restrict__ box,
                                                           const int* __restrict__ box_row, float* __restrict__ out,
                                                           float* __restrict__ part_den) {
  __shared__ float lx[LH * LW], lf[LH * LW];
  __shared__ float red[2][NT / 64];
  const int r = blockIdx.y;
  const int64_t HW = static_cast<int64_t>(H) * W;
  const Tile t = tile_of(W);
  stage_logits(x + static_cast<int64_t>(x_row ? x_row[r] : r) * HW, H, W, d, t, lx, lf);
  __syncthreads();
  const uint8_t* br = MODE == 2 ? nullptr : bits + static_cast<int64_t>(t_row ? t_row[r] : r) * HW;
  const float* wr = (MODE == 1 && box) ? box + static_cast<int64_t>(box_row ? box_row[r] : r) * HW : nullptr;
  const int tx = threadIdx.x % TW, ty_base = (threadIdx.x / TW) * PPT;
  float num = 0.f, den = 0.f;
#pragma unroll
  for (int i = 0; i < PPT; ++i) {
    const int ly = ty_base + i, gy = t.ty0 + ly, gx = t.tx0 + tx;
    if (gy >= H || gx >= W) continue;
    const int64_t p = static_cast<int64_t>(gy) * W + gx;
    const int c = (ly + d) * LW + (tx + d);
    const float a = lx[c], fa = lf[c];
    const unsigned bm = MODE == 2 ? 0xffu : br[p];
    const unsigned on = (MODE == 2 ? 0xffu : bm) & neighbours_inside(gy, gx, H, W, d);
    float acc = 0.f;
#pragma unroll
    for (int k = 0; k < 8; ++k) {
      const int q = c + tap_dy(k) * d * LW + tap_dx(k) * d;
      // evaluated for every neighbour and masked by a multiply: straight-line code, no per-tap branches
      // (staged values are finite for finite logits, out-of-image taps read the zero halo)
      const float sk = static_cast<float>((on >> k) & 1u) * pair_term(a, fa, lx[q], lf[q]);
      if (MODE == 2)
        out[(static_cast<int64_t>(r) * 8 + k) * HW + p] = sk;
      else
        acc += sk;
    }
    if (MODE == 0) out[static_cast<int64_t>(r) * HW + p] = acc;
    if (MODE == 1) {
      const float w = wr ? wr[p] : 1.f;
      num += w * acc;
      den += w * static_cast<float>(__popc(bm));
    }
  }
  if (MODE == 1) {
    num = wave_sum(num);
    den = wave_sum(den);
    if ((threadIdx.x & 63) == 0) {
      red[0][threadIdx.x >> 6] = num;
      red[1][threadIdx.x >> 6] = den;
    }
    __syncthreads();
    if (threadIdx.x == 0) {
      float n = 0.f, e = 0.f;
      for (int i = 0; i < NT / 64; ++i) {
        n += red[0][i];
        e += red[1][i];
      }
      out[static_cast<int64_t>(r) * gridDim.x + blockIdx.x] = n;
      part_den[static_cast<int64_t>(r) * gridDim.x + blockIdx.x] = e;
    }
  }
}

// The matcher's whole per-mask pass in one read of the mask logits (matcher.py:42-83): for row r (query q
// of image b = img[r]) and this tile,
//   part_cost[r, tile, g] = sum_p box[b, g, p] sum_k bit_k(p) s_k(p)      g < gcount[b]  (0 for g >= it)
//   rowmax[r, y, tile_x]  = max over the tile's columns of x (the W-axis projection)
//   colmax[r, tile_y, x]  = max over the tile's rows of x    (the H-axis projection)
constexpr int kMaxG = 256;
__global__ void __launch_bounds__(NT) match_cost_kernel(const float* __restrict__ x, int H, int W, int d, int Q,
                                                        const uint8_t* __restrict__ bits, const float* __restrict__ box,
                                                        const int* __restrict__ gcount, const int* __restrict__ gbox,
                                                        int Gm, float* __restrict__ part_cost, float* __restrict__ rowmax,
                                                        float* __restrict__ colmax) {
  __shared__ float lx[LH * LW], lf[LH * LW];
  __shared__ float red[NT / 64][kMaxG];
  __shared__ float cmax[NT / 64][TW];
  const int r = blockIdx.y, b = r / Q;
  const int64_t HW = static_cast<int64_t>(H) * W;
  const Tile t = tile_of(W);
  const int ntx = (W + TW - 1) / TW, nty = (H + TH - 1) / TH;
  stage_logits(x + static_cast<int64_t>(r) * HW, H, W, d, t, lx, lf);
  __syncthreads();
  const uint8_t* br = bits + static_cast<int64_t>(b) * HW;
  const int tx = threadIdx.x % TW, wave = threadIdx.x / TW, ty_base = wave * PPT;
  const int gx = t.tx0 + tx;
  float A[PPT];
  int64_t P[PPT];
  float cm = -INFINITY;
#pragma unroll
  for (int i = 0; i < PPT; ++i) {
    const int ly = ty_base + i, gy = t.ty0 + ly;
    A[i] = 0.f;
    P[i] = -1;
    float rv = -INFINITY;
    if (gy < H && gx < W) {
      const int64_t p = static_cast<int64_t>(gy) * W + gx;
      P[i] = p;
      const int c = (ly + d) * LW + (tx + d);
      const float a = lx[c], fa = lf[c];
      rv = a;
      cm = fmaxf(cm, a);
      const unsigned on = br[p] & neighbours_inside(gy, gx, H, W, d);
      float acc = 0.f;
#pragma unroll
      for (int k = 0; k < 8; ++k) {
        const int q = c + tap_dy(k) * d * LW + tap_dx(k) * d;
        acc = fmaf(static_cast<float>((on >> k) & 1u), pair_term(a, fa, lx[q], lf[q]), acc);
      }
      A[i] = acc;
    }
    // row max over this wave's 64 columns
    for (int off = 32; off > 0; off >>= 1) rv = fmaxf(rv, __shfl_xor(rv, off));
    if (tx == 0 && gy < H) rowmax[(static_cast<int64_t>(r) * H + gy) * ntx + blockIdx.x % ntx] = rv;
  }
  cmax[wave][tx] = cm;
  // box-weighted sums, one wave reduction per target whose nonzero bounding box meets this tile
  const int G = gcount[b];
  const float* bb = box + static_cast<int64_t>(b) * Gm * HW;
  for (int g = 0; g < G; ++g) {
    const int* bx = gbox + (static_cast<int64_t>(b) * Gm + g) * 4;  // [y0, y1) x [x0, x1)
    if (bx[0] >= min(t.ty0 + TH, H) || bx[1] <= t.ty0 || bx[2] >= min(t.tx0 + TW, W) || bx[3] <= t.tx0) {
      if (threadIdx.x % TW == 0) red[wave][g] = 0.f;
      continue;
    }
    const float* bg = bb + static_cast<int64_t>(g) * HW;
    float v = 0.f;
#pragma unroll
    for (int i = 0; i < PPT; ++i)
      if (P[i] >= 0) v += A[i] * bg[P[i]];
    v = wave_sum(v);
    if (tx == 0) red[wave][g] = v;
  }
  __syncthreads();
  float* pc = part_cost + (static_cast<int64_t>(r) * gridDim.x + blockIdx.x) * Gm;
  for (int g = threadIdx.x; g < Gm; g += NT) {
    float v = 0.f;
    if (g < G)
      for (int w = 0; w < NT / 64; ++w) v += red[w][g];
    pc[g] = v;
  }
  if (threadIdx.x < TW && gx < W) {
    float m = cmax[0][threadIdx.x];
    for (int w = 1; w < NT / 64; ++w) m = fmaxf(m, cmax[w][threadIdx.x]);
    colmax[(static_cast<int64_t>(r) * nty + blockIdx.x / ntx) * W + gx] = m;
  }
}

// grad_x[r, p] = g[r] * sum_k D(x_p, x_q) (w(p) bit_k(p) + w(q) bit_{7-k}(q)),  q = p + off_k in the image
__global__ void __launch_bounds__(NT) pairwise_bwd_kernel(const float* __restrict__ x, const int* __restrict__ x_row,
                                                          int H, int W, int d, const uint8_t* __restrict__ bits,
                                                          const int* __restrict__ t_row, const float* __restrict__ box,
                                                          const int* __restrict__ box_row, const float* __restrict__ g,
                                                          float* __restrict__ grad) {
  __shared__ float lx[LH * LW], lw[LH * LW];
  __shared__ uint8_t lbits[LH * LW];
  const int r = blockIdx.y;
  const int64_t HW = static_cast<int64_t>(H) * W;
  const Tile t = tile_of(W);
  const float* xr = x + static_cast<int64_t>(x_row ? x_row[r] : r) * HW;
  const uint8_t* br = bits + static_cast<int64_t>(t_row ? t_row[r] : r) * HW;
  const float* wr = box ? box + static_cast<int64_t>(box_row ? box_row[r] : r) * HW : nullptr;
  const int hh = TH + 2 * d, ww = TW + 2 * d;
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  for (int yy = wave; yy < hh; yy += NT / 64) {
    for (int xx = lane; xx < ww; xx += 64) {
      const int gy = t.ty0 - d + yy, gx = t.tx0 - d + xx;
      uint8_t bv = 0;
      float w = 0.f, v = 0.f;
      if (inside(gy, gx, H, W)) {
        const int64_t p = static_cast<int64_t>(gy) * W + gx;
        v = xr[p];
        bv = br[p];
        w = wr ? wr[p] : 1.f;
      }
      lx[yy * LW + xx] = v;
      lbits[yy * LW + xx] = bv;
      lw[yy * LW + xx] = w;
    }
  }
  __syncthreads();
  const float gr = g[r];
  const int tx = threadIdx.x % TW, ty_base = (threadIdx.x / TW) * PPT;
#pragma unroll
  for (int i = 0; i < PPT; ++i) {
    const int ly = ty_base + i, gy = t.ty0 + ly, gx = t.tx0 + tx;
    if (gy >= H || gx >= W) continue;
    const int c = (ly + d) * LW + (tx + d);
    const float a = lx[c], wc = lw[c];
    const float sna = sigmoid_neg(a);
    const unsigned bc = lbits[c];
    float acc = 0.f;
#pragma unroll
    for (int k = 0; k < 8; ++k) {
      const int dy = tap_dy(k) * d, dx = tap_dx(k) * d;
      if (!inside(gy + dy, gx + dx, H, W)) continue;
      const int q = c + dy * LW + dx;
      // the centre's own term k, and the neighbour's mirrored term 7-k (which reads x_p as its neighbour)
      float wt = ((bc >> k) & 1u) ? wc : 0.f;
      if ((lbits[q] >> (7 - k)) & 1u) wt += lw[q];
      if (wt != 0.f) acc += wt * pair_grad(a, sna, lx[q]);
    }
    grad[static_cast<int64_t>(r) * HW + static_cast<int64_t>(gy) * W + gx] = gr * acc;
  }
}

// bits[n, p] = sum_k (sim[n, k, p] >= thr) << k
__global__ void threshold_bits_kernel(const float* __restrict__ sim, int64_t HW, int64_t total, float thr,
                                      uint8_t* __restrict__ bits) {
  const int64_t i = blockIdx.x * static_cast<int64_t>(blockDim.x) + threadIdx.x;
  if (i >= total) return;
  const int64_t n = i / HW, p = i % HW;
  const float* s = sim + n * 8 * HW + p;
  unsigned b = 0;
#pragma unroll
  for (int k = 0; k < 8; ++k) b |= (s[k * HW] >= thr ? 1u : 0u) << k;
  bits[i] = static_cast<uint8_t>(b);
}

// ---- target preparation ----------------------------------------------------------------------------
// skimage.color.rgb2lab (D65, 2 degree observer) on img_as_float(uint8), computed in double as skimage does
__device__ void rgb2lab(double r, double g, double b, double* lab) {
  auto lin = [](double c) { return c > 0.04045 ? pow((c + 0.055) / 1.055, 2.4) : c / 12.92; };
  r = lin(r);
  g = lin(g);
  b = lin(b);
  // xyz_from_rgb (sRGB primaries, D65)
  double X = 0.412453 * r + 0.357580 * g + 0.180423 * b;
  double Y = 0.212671 * r + 0.715160 * g + 0.072169 * b;
  double Z = 0.019334 * r + 0.119193 * g + 0.950227 * b;
  X /= 0.95047;
  Z /= 1.08883;
  auto f = [](double t) { return t > 0.008856 ? cbrt(t) : 7.787 * t + 16.0 / 116.0; };
  const double fx = f(X), fy = f(Y), fz = f(Z);
  lab[0] = 116.0 * fy - 16.0;
  lab[1] = 500.0 * (fx - fy);
  lab[2] = 200.0 * (fy - fz);
}

// images (B, 3, Hp, Wp) float (0..255, zero padded) -> lab (B, 3, Hp/s, Wp/s): avg_pool s x s, .byte(), rgb2lab
__global__ void weaksup_lab_kernel(const float* __restrict__ img, int B, int Hp, int Wp, int s,
                                   float* __restrict__ lab) {
  const int h = Hp / s, w = Wp / s;
  const int64_t i = blockIdx.x * static_cast<int64_t>(blockDim.x) + threadIdx.x;
  if (i >= static_cast<int64_t>(B) * h * w) return;
  const int b = static_cast<int>(i / (static_cast<int64_t>(h) * w));
  const int y = static_cast<int>((i / w) % h), xcol = static_cast<int>(i % w);
  double rgb[3];
  for (int ch = 0; ch < 3; ++ch) {
    const float* src = img + ((static_cast<int64_t>(b) * 3 + ch) * Hp + static_cast<int64_t>(y) * s) * Wp +
                       static_cast<int64_t>(xcol) * s;
    float acc = 0.f;
    for (int dy = 0; dy < s; ++dy)
      for (int dx = 0; dx < s; ++dx) acc += src[static_cast<int64_t>(dy) * Wp + dx];
    const float avg = acc / static_cast<float>(s * s);
    // Tensor.byte(): float -> uint8 truncates toward zero (inputs are in [0, 255])
    const int u8 = static_cast<int>(fminf(fmaxf(avg, 0.f), 255.f));
    rgb[ch] = static_cast<double>(u8) / 255.0;
  }
  double o[3];
  rgb2lab(rgb[0], rgb[1], rgb[2], o);
  const int64_t plane = static_cast<int64_t>(h) * w;
  for (int ch = 0; ch < 3; ++ch)
    lab[(static_cast<int64_t>(b) * 3 + ch) * plane + static_cast<int64_t>(y) * w + xcol] = static_cast<float>(o[ch]);
}

// sim[b, k, p] = exp(-||lab_p - lab_q|| * 0.5) * mask_q over q = p + d*off_k (zero outside the image)
__global__ void color_similarity_kernel(const float* __restrict__ lab, const float* __restrict__ mask, int B, int h,
                                        int w, int d, float* __restrict__ sim) {
  const int64_t i = blockIdx.x * static_cast<int64_t>(blockDim.x) + threadIdx.x;
  const int64_t plane = static_cast<int64_t>(h) * w;
  if (i >= B * plane) return;
  const int b = static_cast<int>(i / plane);
  const int64_t p = i % plane;
  const int y = static_cast<int>(p / w), x0 = static_cast<int>(p % w);
  const float* L = lab + static_cast<int64_t>(b) * 3 * plane;
  const float l0 = L[p], a0 = L[plane + p], b0 = L[2 * plane + p];
#pragma unroll
  for (int k = 0; k < 8; ++k) {
    const int yy = y + tap_dy(k) * d, xx = x0 + tap_dx(k) * d;
    float l1 = 0.f, a1 = 0.f, b1 = 0.f, m = 0.f;
    if (yy >= 0 && yy < h && xx >= 0 && xx < w) {
      const int64_t q = static_cast<int64_t>(yy) * w + xx;
      l1 = L[q];
      a1 = L[plane + q];
      b1 = L[2 * plane + q];
      m = mask[static_cast<int64_t>(b) * plane + q];
    }
    const float dl = l0 - l1, da = a0 - a1, db = b0 - b1;
    const float nrm = sqrtf(dl * dl + da * da + db * db);
    sim[(static_cast<int64_t>(b) * 8 + k) * plane + p] = expf(-nrm * 0.5f) * m;
  }
}

int check_rows(const char* fn, const void* x, int R, int H, int W, int d) {
  if (R < 0 || H < 0 || W < 0 || (R > 0 && !x)) return m2f::fail(M2F_EINVAL, "%s: bad arguments", fn);
  if (d < 1 || d > kMaxDil) return m2f::fail(M2F_EUNSUPPORTED, "%s: dilation %d not in [1, %d]", fn, d, kMaxDil);
  if (R > 65535) return m2f::fail(M2F_EUNSUPPORTED, "%s: %d rows > 65535", fn, R);
  return M2F_OK;
}

unsigned n_tiles(int H, int W) { return m2f::ceil_div(H, TH) * m2f::ceil_div(W, TW); }

}  // namespace

extern "C" int m2f_pairwise_tiles(int H, int W) { return static_cast<int>(n_tiles(H, W)); }

extern "C" int m2f_pairwise_rows(const float* x, const int* x_row, int R, int H, int W, int dilation,
                                 const uint8_t* bits, const int* t_row, const float* box, const int* box_row, int mode,
                                 float* out, float* out_den, void* stream) {
  const char* fn = "m2f_pairwise_rows";
  if (int e = check_rows(fn, x, R, H, W, dilation)) return e;
  if (mode < 0 || mode > 2 || !out || (mode != 2 && !bits) || (mode == 1 && !out_den))
    return m2f::fail(M2F_EINVAL, "%s: bad mode/outputs", fn);
  if (R == 0 || H == 0 || W == 0) return m2f::ok();
  const dim3 grid(n_tiles(H, W), R);
  hipStream_t st = static_cast<hipStream_t>(stream);
  if (mode == 0)
    pairwise_rows_kernel<0><<<grid, NT, 0, st>>>(x, x_row, H, W, dilation, bits, t_row, box, box_row, out, out_den);
  else if (mode == 1)
    pairwise_rows_kernel<1><<<grid, NT, 0, st>>>(x, x_row, H, W, dilation, bits, t_row, box, box_row, out, out_den);
  else
    pairwise_rows_kernel<2><<<grid, NT, 0, st>>>(x, x_row, H, W, dilation, bits, t_row, box, box_row, out, out_den);
  return m2f::check_launch(fn);
}

extern "C" int m2f_pairwise_match_cost(const float* x, int B, int Q, int H, int W, int dilation, const uint8_t* bits,
                                       const float* box, const int* gcount, const int* gbox, int Gm, float* part_cost,
                                       float* rowmax, float* colmax, void* stream) {
  const char* fn = "m2f_pairwise_match_cost";
  if (int e = check_rows(fn, x, B * Q, H, W, dilation)) return e;
  if (Gm < 0 || Gm > kMaxG) return m2f::fail(M2F_EUNSUPPORTED, "%s: %d targets > %d", fn, Gm, kMaxG);
  if (B * Q > 0 && H > 0 && W > 0 && (!bits || !gcount || !rowmax || !colmax || (Gm > 0 && (!box || !gbox || !part_cost))))
    return m2f::fail(M2F_EINVAL, "%s: bad arguments", fn);
  if (B * Q == 0 || H == 0 || W == 0) return m2f::ok();
  match_cost_kernel<<<dim3(n_tiles(H, W), B * Q), NT, 0, static_cast<hipStream_t>(stream)>>>(
      x, H, W, dilation, Q, bits, box, gcount, gbox, Gm, part_cost, rowmax, colmax);
  return m2f::check_launch(fn);
}

extern "C" int m2f_pairwise_rows_bwd(const float* x, const int* x_row, int R, int H, int W, int dilation,
                                     const uint8_t* bits, const int* t_row, const float* box, const int* box_row,
                                     const float* grad_scale, float* grad, void* stream) {
  const char* fn = "m2f_pairwise_rows_bwd";
  if (int e = check_rows(fn, x, R, H, W, dilation)) return e;
  if (R > 0 && (!bits || !grad_scale || !grad)) return m2f::fail(M2F_EINVAL, "%s: bad arguments", fn);
  if (R == 0 || H == 0 || W == 0) return m2f::ok();
  pairwise_bwd_kernel<<<dim3(n_tiles(H, W), R), NT, 0, static_cast<hipStream_t>(stream)>>>(
      x, x_row, H, W, dilation, bits, t_row, box, box_row, grad_scale, grad);
  return m2f::check_launch(fn);
}

extern "C" int m2f_threshold_bits(const float* sim, int N, int64_t HW, float thr, uint8_t* bits, void* stream) {
  const char* fn = "m2f_threshold_bits";
  if (N < 0 || HW < 0 || (N > 0 && HW > 0 && (!sim || !bits))) return m2f::fail(M2F_EINVAL, "%s: bad arguments", fn);
  const int64_t total = static_cast<int64_t>(N) * HW;
  if (total == 0) return m2f::ok();
  threshold_bits_kernel<<<m2f::ceil_div(total, 256), 256, 0, static_cast<hipStream_t>(stream)>>>(sim, HW, total, thr,
                                                                                                 bits);
  return m2f::check_launch(fn);
}

extern "C" int m2f_weaksup_lab(const float* images, int B, int Hp, int Wp, int stride, float* lab, void* stream) {
  const char* fn = "m2f_weaksup_lab";
  if (B < 0 || Hp < 0 || Wp < 0 || stride < 1 || Hp % stride || Wp % stride || (B > 0 && (!images || !lab)))
    return m2f::fail(M2F_EINVAL, "%s: bad arguments (H, W must be multiples of the stride)", fn);
  const int64_t total = static_cast<int64_t>(B) * (Hp / stride) * (Wp / stride);
  if (total == 0) return m2f::ok();
  weaksup_lab_kernel<<<m2f::ceil_div(total, 256), 256, 0, static_cast<hipStream_t>(stream)>>>(images, B, Hp, Wp,
                                                                                             stride, lab);
  return m2f::check_launch(fn);
}

extern "C" int m2f_color_similarity(const float* lab, const float* mask, int B, int h, int w, int dilation, float* sim,
                                    void* stream) {
  const char* fn = "m2f_color_similarity";
  if (B < 0 || h < 0 || w < 0 || dilation < 1 || (B > 0 && (!lab || !mask || !sim)))
    return m2f::fail(M2F_EINVAL, "%s: bad arguments", fn);
  const int64_t total = static_cast<int64_t>(B) * h * w;
  if (total == 0) return m2f::ok();
  color_similarity_kernel<<<m2f::ceil_div(total, 256), 256, 0, static_cast<hipStream_t>(stream)>>>(lab, mask, B, h, w,
                                                                                                  dilation, sim);
  return m2f::check_launch(fn);
}
