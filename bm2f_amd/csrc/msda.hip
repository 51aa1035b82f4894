// Multi-scale deformable attention (MSDA) forward / backward for gfx950.
//
// Semantics follow the reference op exactly (mask2former/modeling/pixel_decoder/ops):
//   * sampling point:  h = loc_y * H_l - 0.5, w = loc_x * W_l - 0.5; the point contributes only if
//     -1 < h < H_l and -1 < w < W_l (ms_deform_im2col_cuda.cuh:290-296);
//   * bilinear with per-corner zero padding, value = w1*v1 + w2*v2 + w3*v3 + w4*v4 (.cuh:38-89);
//   * backward: grad_value[corner] += w_corner * g * a; grad_attn = sum_c g * val;
//     grad_loc = (W * sum_c dval/dw * g * a, H * sum_c dval/dh * g * a)  (.cuh:92-164).
//
// Layout choices (MI355X-first, not the reference's thread-per-channel/1024-thread blocks):
//   * fp32 fast path: a pair (n, q, m) is served by G = D/4 lanes, each owning 4 consecutive
//     channels (one float4).  A wave64 therefore handles 64/G pairs; for D = 32 that is the 8 heads
//     of one query, every corner fetch is one 128-byte row per pair, and the channel reductions of
//     the backward are an in-lane sum of 4 followed by log2(G) xor-shuffles (no LDS, no barriers).
//   * the backward's grad_value scatter is the costly part (one 128-B row add per corner per
//     point).  With host spatial shapes and Lq == S (the encoder), queries are grouped into spatial
//     tiles and the adds go to a per-workgroup LDS window of the sampled neighbourhood, flushed to
//     HBM once with row-contiguous atomics; samples falling outside the window take the direct path.
//   * fp64 and channel counts the fast path does not cover use straightforward generic kernels.
#include "common.h"
#include "msda_device.h"

#include <algorithm>
#include <atomic>
#include <cmath>
#include <cstdlib>
#include <cstring>
#include <type_traits>

namespace m2f {
std::string& last_error() {
  static thread_local std::string s;
  return s;
}
}  // namespace m2f

extern "C" const char* m2f_last_error(void) { return m2f::last_error().c_str(); }
extern "C" int m2f_abi_version(void) { return 1; }

namespace {
constexpr const char* kOptionNames[m2f::kOptCount] = {
    "msda_threads", "msda_tile", "msda_tile_w", "msda_halo", "msda_win_rows", "msda_bwd_tiled", "msda_fwd_tiled",
    "mattn_dq_atomic", "gemm_nt_cfg", "x3_tn_nw", "x3_tn_blocks", "x3_nt_cfg", "msda_fwd_quad", "msda_bwd_overlap",
    "msda_bwd_det", "msda_fwd_pb", "msda_bwd_ratio", "msda_fwd_lds", "msda_fwd_tile", "msda_fwd_tile_w",
    "msda_fwd_cap", "msda_fwd_halo", "mattn_fwd_minblk", "mattn_bwd_minblk", "mask_df_stage",
    "mattn_bwd_keys", "mattn_xcd", "mattn_combine", "msda_bwd_rowsort", "msda_bwd_walk4", "msda_fwd_xcd", "msda_fwd_pair"};
std::atomic<int64_t> g_options[m2f::kOptCount] = {};
struct OptionInit {
  OptionInit() {
    for (auto& o : g_options) o.store(-1);
  }
} g_option_init;

int option_index(const char* name) {
  for (int i = 0; name && i < m2f::kOptCount; ++i)
    if (std::strcmp(name, kOptionNames[i]) == 0) return i;
  return -1;
}
}  // namespace

int64_t m2f::option_raw(Option o) { return g_options[o].load(std::memory_order_relaxed); }

extern "C" int m2f_set_option(const char* name, int64_t value) {
  const int i = option_index(name);
  if (i < 0) return m2f::fail(M2F_EINVAL, "m2f_set_option: unknown option '%s'", name ? name : "(null)");
  g_options[i].store(value < 0 ? -1 : value);
  return m2f::ok();
}

extern "C" int m2f_get_option(const char* name, int64_t* value) {
  const int i = option_index(name);
  if (i < 0 || !value) return m2f::fail(M2F_EINVAL, "m2f_get_option: unknown option '%s'", name ? name : "(null)");
  *value = g_options[i].load();
  return m2f::ok();
}

namespace {

using namespace m2f_msda;

constexpr int kMaxLevels = 16;

// ------------------------------------------------------------------------------------------------
// Generic kernels (any channel count, float or double).  Thread per output element for the forward,
// block per (n, q, m) pair for the backward.
// ------------------------------------------------------------------------------------------------

template <typename T>
__device__ __forceinline__ T bilinear_gather(const T* __restrict__ v, int H, int W, int64_t rs, T h, T w) {
  const int h0 = static_cast<int>(floor(h));
  const int w0 = static_cast<int>(floor(w));
  const T lh = h - h0, lw = w - w0;
  const T hh = T(1) - lh, hw = T(1) - lw;
  T v1 = 0, v2 = 0, v3 = 0, v4 = 0;
  if (h0 >= 0 && w0 >= 0) v1 = v[(static_cast<int64_t>(h0) * W + w0) * rs];
  if (h0 >= 0 && w0 + 1 <= W - 1) v2 = v[(static_cast<int64_t>(h0) * W + w0 + 1) * rs];
  if (h0 + 1 <= H - 1 && w0 >= 0) v3 = v[(static_cast<int64_t>(h0 + 1) * W + w0) * rs];
  if (h0 + 1 <= H - 1 && w0 + 1 <= W - 1) v4 = v[(static_cast<int64_t>(h0 + 1) * W + w0 + 1) * rs];
  const T w1 = hh * hw, w2 = hh * lw, w3 = lh * hw, w4 = lh * lw;
  return w1 * v1 + w2 * v2 + w3 * v3 + w4 * v4;
}

template <typename T>
__global__ void __launch_bounds__(256) msda_fwd_generic(
    const T* __restrict__ value, const int64_t* __restrict__ shapes, const int64_t* __restrict__ lsi,
    const T* __restrict__ loc, const T* __restrict__ attn, int64_t total, int S, int M, int D, int L,
    int Lq, int P, T* __restrict__ out) {
  const int64_t rs = static_cast<int64_t>(M) * D;
  for (int64_t idx = blockIdx.x * static_cast<int64_t>(blockDim.x) + threadIdx.x; idx < total;
       idx += static_cast<int64_t>(gridDim.x) * blockDim.x) {
    const int c = static_cast<int>(idx % D);
    const int64_t pair = idx / D;
    const int m = static_cast<int>(pair % M);
    const int64_t n = pair / M / Lq;
    const T* vb = value + (n * S * M + m) * D + c;
    const T* lp = loc + pair * L * P * 2;
    const T* ap = attn + pair * L * P;
    T col = 0;
    for (int l = 0; l < L; ++l) {
      const int H = static_cast<int>(shapes[2 * l]);
      const int W = static_cast<int>(shapes[2 * l + 1]);
      const T* vl = vb + lsi[l] * rs;
      for (int p = 0; p < P; ++p, lp += 2, ++ap) {
        const T h = lp[1] * H - T(0.5);
        const T w = lp[0] * W - T(0.5);
        if (h > T(-1) && w > T(-1) && h < T(H) && w < T(W))
          col += bilinear_gather(vl, H, W, rs, h, w) * ap[0];
      }
    }
    out[idx] = col;
  }
}

template <typename T, int BS>
__device__ __forceinline__ T block_sum(T v, T* red) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o);
  const int wid = threadIdx.x >> 6;
  if ((threadIdx.x & 63) == 0) red[wid] = v;
  __syncthreads();
  T s = 0;
#pragma unroll
  for (int i = 0; i < BS / 64; ++i) s += red[i];
  __syncthreads();
  return s;
}

template <typename T, int BS>
__global__ void __launch_bounds__(BS) msda_bwd_generic(
    const T* __restrict__ value, const int64_t* __restrict__ shapes, const int64_t* __restrict__ lsi,
    const T* __restrict__ loc, const T* __restrict__ attn, const T* __restrict__ gout, int S, int M, int D,
    int L, int Lq, int P, T* __restrict__ gvalue, T* __restrict__ gloc, T* __restrict__ gattn) {
  __shared__ T red[3][BS / 64];
  const int64_t pair = blockIdx.x;
  const int m = static_cast<int>(pair % M);
  const int64_t n = pair / M / Lq;
  const int64_t rs = static_cast<int64_t>(M) * D;
  const int64_t vbase = (n * S * M + m) * D;
  const T* go = gout + pair * D;
  for (int l = 0; l < L; ++l) {
    const int H = static_cast<int>(shapes[2 * l]);
    const int W = static_cast<int>(shapes[2 * l + 1]);
    const int64_t lbase = vbase + lsi[l] * rs;
    for (int p = 0; p < P; ++p) {
      const int64_t k = (pair * L + l) * P + p;
      const T lw = loc[2 * k], lh = loc[2 * k + 1], a = attn[k];
      const T h = lh * H - T(0.5), w = lw * W - T(0.5);
      const bool ok = h > T(-1) && w > T(-1) && h < T(H) && w < T(W);
      T pa = 0, px = 0, py = 0;
      if (ok) {  // uniform across the block
        const int h0 = static_cast<int>(floor(h)), w0 = static_cast<int>(floor(w));
        const T lh_ = h - h0, lw_ = w - w0, hh = T(1) - lh_, hw = T(1) - lw_;
        const T w1 = hh * hw, w2 = hh * lw_, w3 = lh_ * hw, w4 = lh_ * lw_;
        const bool c1 = h0 >= 0 && w0 >= 0, c2 = h0 >= 0 && w0 + 1 <= W - 1;
        const bool c3 = h0 + 1 <= H - 1 && w0 >= 0, c4 = h0 + 1 <= H - 1 && w0 + 1 <= W - 1;
        const int64_t o1 = lbase + (static_cast<int64_t>(h0) * W + w0) * rs;
        const int64_t o2 = o1 + rs, o3 = o1 + static_cast<int64_t>(W) * rs, o4 = o3 + rs;
        for (int c = threadIdx.x; c < D; c += BS) {
          const T g = go[c];
          const T tg = g * a;
          T gh = 0, gw = 0, v1 = 0, v2 = 0, v3 = 0, v4 = 0;
          if (c1) { v1 = value[o1 + c]; gh -= hw * v1; gw -= hh * v1; atomicAdd(gvalue + o1 + c, w1 * tg); }
          if (c2) { v2 = value[o2 + c]; gh -= lw_ * v2; gw += hh * v2; atomicAdd(gvalue + o2 + c, w2 * tg); }
          if (c3) { v3 = value[o3 + c]; gh += hw * v3; gw -= lh_ * v3; atomicAdd(gvalue + o3 + c, w3 * tg); }
          if (c4) { v4 = value[o4 + c]; gh += lw_ * v4; gw += lh_ * v4; atomicAdd(gvalue + o4 + c, w4 * tg); }
          pa += g * (w1 * v1 + w2 * v2 + w3 * v3 + w4 * v4);
          px += W * gw * tg;
          py += H * gh * tg;
        }
      }
      pa = block_sum<T, BS>(pa, red[0]);
      px = block_sum<T, BS>(px, red[1]);
      py = block_sum<T, BS>(py, red[2]);
      if (threadIdx.x == 0) {
        gattn[k] = pa;
        gloc[2 * k] = px;
        gloc[2 * k + 1] = py;
      }
    }
  }
}

template <int D, int PT>
__global__ void __launch_bounds__(256) msda_fwd_f32_vec(
    const float* __restrict__ value, const int64_t* __restrict__ shapes, const int64_t* __restrict__ lsi,
    const float* __restrict__ loc, const float* __restrict__ attn, int64_t npairs, int S, int M, int L,
    int Lq, int Prt, float* __restrict__ out) {
  constexpr int G = D / 4;
  const int P = PT > 0 ? PT : Prt;
  __shared__ int sH[kMaxLevels], sW[kMaxLevels];
  __shared__ int64_t sSt[kMaxLevels];
  if (threadIdx.x < L) {
    sH[threadIdx.x] = static_cast<int>(shapes[2 * threadIdx.x]);
    sW[threadIdx.x] = static_cast<int>(shapes[2 * threadIdx.x + 1]);
    sSt[threadIdx.x] = lsi[threadIdx.x];
  }
  __syncthreads();
  const int64_t pair = static_cast<int64_t>(blockIdx.x) * (256 / G) + threadIdx.x / G;
  if (pair >= npairs) return;
  const int j = threadIdx.x % G;
  const int m = static_cast<int>(pair % M);
  const int64_t n = pair / M / Lq;
  const int64_t rs = static_cast<int64_t>(M) * D;
  const int64_t vbase = (n * S * M + m) * D + 4 * j;
  const float* lp = loc + pair * L * P * 2;
  const float* ap = attn + pair * L * P;
  f4 acc = {0.f, 0.f, 0.f, 0.f};
  for (int l = 0; l < L; ++l) {
    const int H = sH[l], W = sW[l];
    const int64_t lbase = vbase + sSt[l] * rs;
#pragma unroll
    for (int p = 0; p < P; ++p) {
      const int kk = l * P + p;
      const float2 xy = *reinterpret_cast<const float2*>(lp + 2 * kk);
      const float a = ap[kk];
      const Corners k = make_corners(xy.x, xy.y, H, W, lbase, rs);
      const f4 v1 = ld4(value + k.o1), v2 = ld4(value + k.o2), v3 = ld4(value + k.o3), v4 = ld4(value + k.o4);
      const f4 z = {0.f, 0.f, 0.f, 0.f};
      const f4 u1 = k.c1 ? v1 : z, u2 = k.c2 ? v2 : z, u3 = k.c3 ? v3 : z, u4 = k.c4 ? v4 : z;
      const f4 val = k.w1 * u1 + k.w2 * u2 + k.w3 * u3 + k.w4 * u4;
      acc += k.ok ? val * a : z;
    }
  }
  *reinterpret_cast<f4*>(out + pair * D + 4 * j) = acc;
}

// Backward, direct-atomic variant: every corner contribution goes straight to HBM.
template <int D, int PT>
__global__ void __launch_bounds__(256) msda_bwd_f32_vec(
    const float* __restrict__ value, const int64_t* __restrict__ shapes, const int64_t* __restrict__ lsi,
    const float* __restrict__ loc, const float* __restrict__ attn, const float* __restrict__ gout,
    int64_t npairs, int S, int M, int L, int Lq, int Prt, float* __restrict__ gvalue,
    float* __restrict__ gloc, float* __restrict__ gattn) {
  constexpr int G = D / 4;
  const int P = PT > 0 ? PT : Prt;
  __shared__ int sH[kMaxLevels], sW[kMaxLevels];
  __shared__ int64_t sSt[kMaxLevels];
  if (threadIdx.x < L) {
    sH[threadIdx.x] = static_cast<int>(shapes[2 * threadIdx.x]);
    sW[threadIdx.x] = static_cast<int>(shapes[2 * threadIdx.x + 1]);
    sSt[threadIdx.x] = lsi[threadIdx.x];
  }
  __syncthreads();
  const int64_t pair = static_cast<int64_t>(blockIdx.x) * (256 / G) + threadIdx.x / G;
  if (pair >= npairs) return;
  const int j = threadIdx.x % G;
  const int m = static_cast<int>(pair % M);
  const int64_t n = pair / M / Lq;
  const int64_t rs = static_cast<int64_t>(M) * D;
  const int64_t vbase = (n * S * M + m) * D + 4 * j;
  const f4 g = ld4(gout + pair * D + 4 * j);
  const f4 z = {0.f, 0.f, 0.f, 0.f};
  for (int l = 0; l < L; ++l) {
    const int H = sH[l], W = sW[l];
    const int64_t lbase = vbase + sSt[l] * rs;
#pragma unroll
    for (int p = 0; p < P; ++p) {
      const int64_t kk = (pair * L + l) * P + p;
      const float2 xy = *reinterpret_cast<const float2*>(loc + 2 * kk);
      const float a = attn[kk];
      const Corners k = make_corners(xy.x, xy.y, H, W, lbase, rs);
      f4 v1 = ld4(value + k.o1), v2 = ld4(value + k.o2), v3 = ld4(value + k.o3), v4 = ld4(value + k.o4);
      v1 = k.c1 ? v1 : z; v2 = k.c2 ? v2 : z; v3 = k.c3 ? v3 : z; v4 = k.c4 ? v4 : z;
      const f4 tg = g * a;
      const f4 val = k.w1 * v1 + k.w2 * v2 + k.w3 * v3 + k.w4 * v4;
      // d val / d w and d val / d h per channel, in the reference's accumulation order (.cuh:125-157)
      const f4 gw = -k.hy * v1 + k.hy * v2 - k.ly * v3 + k.ly * v4;
      const f4 gh = -k.hx * v1 - k.lx * v2 + k.hx * v3 + k.lx * v4;
      const f4 ta = g * val, tx = gw * tg, ty = gh * tg;
      float pa = ta.x + ta.y + ta.z + ta.w;
      float px = tx.x + tx.y + tx.z + tx.w;
      float py = ty.x + ty.y + ty.z + ty.w;
#pragma unroll
      for (int o = G / 2; o > 0; o >>= 1) {
        pa += __shfl_xor(pa, o);
        px += __shfl_xor(px, o);
        py += __shfl_xor(py, o);
      }
      if (k.ok) {
        float* gv = gvalue;
        if (k.c1) { const f4 c = k.w1 * tg; atomicAdd(gv + k.o1, c.x); atomicAdd(gv + k.o1 + 1, c.y); atomicAdd(gv + k.o1 + 2, c.z); atomicAdd(gv + k.o1 + 3, c.w); }
        if (k.c2) { const f4 c = k.w2 * tg; atomicAdd(gv + k.o2, c.x); atomicAdd(gv + k.o2 + 1, c.y); atomicAdd(gv + k.o2 + 2, c.z); atomicAdd(gv + k.o2 + 3, c.w); }
        if (k.c3) { const f4 c = k.w3 * tg; atomicAdd(gv + k.o3, c.x); atomicAdd(gv + k.o3 + 1, c.y); atomicAdd(gv + k.o3 + 2, c.z); atomicAdd(gv + k.o3 + 3, c.w); }
        if (k.c4) { const f4 c = k.w4 * tg; atomicAdd(gv + k.o4, c.x); atomicAdd(gv + k.o4 + 1, c.y); atomicAdd(gv + k.o4 + 2, c.z); atomicAdd(gv + k.o4 + 3, c.w); }
      }
      if (j == 0) {
        gattn[kk] = k.ok ? pa : 0.f;
        *reinterpret_cast<float2*>(gloc + 2 * kk) =
            k.ok ? make_float2(W * px, H * py) : make_float2(0.f, 0.f);
      }
    }
  }
}

// ------------------------------------------------------------------------------------------------
// fp32 backward, spatially tiled: encoder self-attention (Lq == S, query i = pyramid position i).
//
// Workgroup = (spatial tile, head m, image n), 512 threads (two per CU).  A tile is the same normalised rectangle on
// every level (level l's tile ty spans rows [ty*H_l/nty, (ty+1)*H_l/nty)), so its queries at every level
// sample the same neighbourhood of every level.
//
// grad_value is a scatter: every (query, sample, corner) adds w_c * a * g[query] (32 channels) to one
// pixel row.  Here it becomes a gather inside the workgroup:
//   phase 0  one lane per (query, level) derives that level's P samples ONCE (softmax and ref + offset /
//            (W, H) on the fused path, or the given loc / attn) into a 16-byte descriptor {ly, lx, a, floors}
//            per sample in LDS (h = loc_y * H - 0.5 = floor + ly ..., the two floors + 2 packed in 16 bits each;
//            floors -2 and fractions 0 when the sample lies outside (-1, H) x (-1, W): every corner outside),
//            stages the tile's grad_output rows (this head) in LDS and takes the bounding box of
//            the touched corners per level (every global load of the phase issued first).  The window = that
//            box clipped to the tile +- halo.
//   phase 1  counting sort of the samples by the window cell of their 2x2 corner block (the window grid
//            extended by one row / column up and left): an LDS counter per cell (returning adds give each
//            sample its rank), a block-wide exclusive scan, and one 32-bit slot per sample (its descriptor
//            index and its query's g-row offset).  Samples whose corners leave the window are flagged instead.
//   phase 2  a lane quad per query (8 channels per lane) gathers each sample's 4 corner rows (texture path),
//            forms the per-corner channel dots with g and writes grad_loc / grad_attn (or d offset / d logit)
//            once per point (quad transpose-reduce).  Flagged samples add their 4 corner rows with atomics.
//   phase 3  a 4-lane group per window pixel reads the 4 slot ranges whose cells cover it ((y,x) ->
//            corner 1 of cell (y,x), corner 2 of (y,x-1), corner 3 of (y-1,x), corner 4 of (y-1,x-1); the
//            row-major cell order makes them two contiguous ranges), accumulating w_c * a * g[query] in fp32 from the LDS descriptors and g rows (8 channels per
//            lane); the wave's 16 rows are transposed through LDS, 8 at a time, so that each atomic
//            instruction adds two whole 128-B rows to HBM.
//   Phases 2 and 3 read nothing the other writes: their units are dealt from one counter, interleaved
//   (OVERLAP), so the texture-bound gather and the LDS-bound walk run at once.
// Summation order (slot order, atomics across workgroups) is not fixed, as in the reference's atomics, except
// in the deterministic mode (DET, below).
// grad_loc / grad_attn (or d offset / d logit) are owned per (q, m) and written once.
//
// FUSED = true: the samples come from the raw projection (offsets | logits) and the reference points, and
// the outputs are the gradients w.r.t. that projection: d offset = d loc / (W, H) = sum_c dval/dloc * g * a
// in pixel units (the level scale cancels) and d logit = a * (d attn - sum_k a_k d attn_k) (softmax
// backward over the pair's L*P logits).
// ------------------------------------------------------------------------------------------------
#ifndef M2F_WALK_LANES
#define M2F_WALK_LANES 4        // phase-3 lanes per window pixel (2: an experiment build, tools/lib)
#endif
constexpr int kWalkLanes = M2F_WALK_LANES;   // phase-3 lanes per window pixel (32 / kWalkLanes channels each)
constexpr int kMaxBwdWaves = 16;
constexpr int kSortSamples = 6144;  // samples per workgroup the counting sort holds in registers (max_qt * L * P)
static_assert(kSortSamples < 65536, "phase 3's slots hold the sample index in 16 bits");
constexpr int kStageFloats = 8 * 32 + 8;  // per wave: 8 rows x 32 channels + 8 row offsets (a flush half)

struct TileState {
  int bb[kTileMaxL][4];  // min y, max y, min x, max x of touched corners (inclusive)
  int wy0[kTileMaxL], wx0[kTileMaxL], wh[kTileMaxL], ww[kTileMaxL];
  int roff[kTileMaxL + 1];   // window pixel offsets per level
  int coff[kTileMaxL + 1];   // extended-cell offsets per level ((wh+1) x (ww+1) cells)
  int qc[kTileMaxL + 1], qy0[kTileMaxL], qx0[kTileMaxL], qw[kTileMaxL];
  int wsum[kMaxBwdWaves];    // block scan
  float iww[kTileMaxL];      // 1 / ww (phase 3's row -> window coordinates)
  int H[kTileMaxL], W[kTileMaxL], start[kTileMaxL];  // the level shapes in LDS: a kernarg array indexed by a
  float invW[kTileMaxL], invH[kTileMaxL];            // per-lane level is a global load per use
  int next_batch;            // phase-3 row batches handed out dynamically
  int rbin[64];              // row sort: rows per record-count bin, then the bins' start positions
};
// the tiled backward's dynamic LDS (<= 156 KB, make_tile_geom) plus this static block within the CU's 160 KB, and
// within the 160 KB - 1 KB the launcher raises the dynamic limit to
static_assert(sizeof(TileState) <= 1024, "TileState must leave the dynamic LDS its 159 KB");

// g rows in LDS: query qi's 16-byte chunk c (float offset)
__device__ __forceinline__ int g_chunk_off(int qi, int c) { return qi * 32 + 4 * c; }

// Fused-front-end inputs (raw projection + reference points).
struct FrontEnd {
  const float* proj;   // (N, Lq, ld): offsets (M, L, P, 2) then logits (M, L*P); hm: per head m a record
                       // [offsets (L, P, 2) | logits (L*P)] (m2f_msda_fused_*_hm_f32); grad_proj alike
  int ld;
  const float* ref;    // (N or broadcast, Lq, L, 2) [x, y]
  int64_t ref_bs;      // batch stride of ref in elements (0 = broadcast)
  int hm;
  // where head m's offsets / logits start in a projection (or grad_proj) row (LP = L * P)
  __device__ __forceinline__ int off0(int m, int LP) const { return hm ? m * 3 * LP : m * LP * 2; }
  __device__ __forceinline__ int lg0(int m, int M, int LP) const { return hm ? m * 3 * LP + 2 * LP : M * LP * 2 + m * LP; }
};

// pyramid position of the tile's query qi (levels in order, rows of the tile's rectangle on each level)
__device__ __forceinline__ int tile_query(const TileState& ts, int qi) {
  int lq = 0;
  while (qi >= ts.qc[lq + 1]) ++lq;
  const int r = qi - ts.qc[lq];
  return ts.start[lq] + (ts.qy0[lq] + r / ts.qw[lq]) * ts.W[lq] + ts.qx0[lq] + r % ts.qw[lq];
}

__device__ __forceinline__ int wave_incl_scan(int v, int lane) {
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) {
    const int t = __shfl_up(v, o);
    v += lane >= o ? t : 0;
  }
  return v;
}

// window cell of a sample whose top-left corner is (h0, w0), or -1 when a corner inside the level lies
// outside the window
__device__ __forceinline__ int window_cell(const TileState& ts, int l, int h0, int w0, int H, int W) {
  const int wy0 = ts.wy0[l], wx0 = ts.wx0[l], wh = ts.wh[l], ww = ts.ww[l];
  const bool ry = (h0 < 0 || (h0 >= wy0 && h0 < wy0 + wh)) && (h0 + 1 > H - 1 || (h0 + 1 >= wy0 && h0 + 1 < wy0 + wh));
  const bool rx = (w0 < 0 || (w0 >= wx0 && w0 < wx0 + ww)) && (w0 + 1 > W - 1 || (w0 + 1 >= wx0 && w0 + 1 < wx0 + ww));
  return (wh > 0 && ry && rx) ? ts.coff[l] + (h0 - wy0 + 1) * (ww + 1) + (w0 - wx0 + 1) : -1;
}

// STAMP (diagnostic builds only, M2F_DIAG): s_memtime at the phase barriers of each workgroup into `stamps`;
// NOFLUSH (diagnostic builds only): phase 3 without its HBM adds, to price them.
// TPB threads per workgroup: 512 (two workgroups per CU, 12x12 tiles; the default) or 1024 (one, 16x16 tiles).
// Fixed-point scale of the deterministic mode: 2^(61 - b - e) with max |grad_output| < 2^e and Lq < 2^b.  A
// grad_value element sums coef * g over samples whose coefficients (bilinear weight * attention weight, each
// <= 1; a query's attention weights per head sum to 1) total at most the image's Lq queries, so every partial
// and the total stay below 2^61; the resolution is max|g| * 2^-(61 - b) absolute (2^-46 at config 2's 21,504
// queries).
__device__ __forceinline__ float det_scale(unsigned maxbits, int Lq) {
  const float B = __uint_as_float(maxbits);
  int e = 0;
  if (B > 0.f) (void)frexpf(B, &e);
  const int b = 32 - __clz(Lq);
  return ldexpf(1.f, min(61 - b - e, 126));
}

// max |g| over finite entries (as the bits of a non-negative float: the unsigned order is the float order) and a
// flag for any non-finite entry: out[0], out[1] (zeroed by the caller)
__global__ void __launch_bounds__(256) msda_det_scale_kernel(const float4* __restrict__ g, int64_t n4,
                                                             unsigned* __restrict__ out) {
  unsigned mx = 0u, nf = 0u;
  for (int64_t i = blockIdx.x * 256LL + threadIdx.x; i < n4; i += static_cast<int64_t>(gridDim.x) * 256) {
    const float4 v = g[i];
    const float a[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      const unsigned b = __float_as_uint(fabsf(a[k]));
      if (b >= 0x7f800000u) nf = 1u;
      else mx = max(mx, b);
    }
  }
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) { mx = max(mx, __shfl_xor(mx, o)); nf |= __shfl_xor(nf, o); }
  if ((threadIdx.x & 63) == 0) {
    atomicMax(out, mx);
    if (nf) atomicOr(out + 1, 1u);
  }
}

// grad_value = fixed-point sum * 2^-k, added to what the non-finite contributions left there in fp32 (zero almost
// everywhere); skipped when the non-finite flag sent the whole kernel down the fp32 atomics
__global__ void __launch_bounds__(256) msda_det_convert_kernel(const long long* __restrict__ acc, int64_t n, int Lq,
                                                               const unsigned* __restrict__ detscale,
                                                               float* __restrict__ gvalue) {
  if (detscale[1] != 0u) return;
  const double inv = 1.0 / static_cast<double>(det_scale(detscale[0], Lq));
  for (int64_t i = blockIdx.x * 256LL + threadIdx.x; i < n; i += static_cast<int64_t>(gridDim.x) * 256)
    gvalue[i] += static_cast<float>(static_cast<double>(acc[i]) * inv);
}

// DET (deterministic mode, m2f_set_option msda_bwd_det): every grad_value contribution leaving a workgroup (the
// window rows, the out-of-window samples) is converted to 64-bit fixed point (scale 2^k from the launch's max
// |grad_output|, DetScale below) and added with integer atomics, whose sum does not depend on their order; the
// slots of each cell are sorted by sample, so a window row's fp32 partial is summed in a fixed order.  A
// conversion pass writes grad_value.  Non-finite grad_output falls back to the fp32 atomics (flag set by the scale
// pass), as the reference's kernel propagates them.
// Occupancy: four waves per SIMD (<= 128 VGPRs; a 1024-thread workgroup needs that) except for four levels, which
// run 512-thread workgroups only, at two waves per SIMD (<= 256 VGPRs): the L = 4 body (the reference module's
// default n_levels, ops/modules/ms_deform_attn.py:35) spilled 3-10 VGPRs at 128.
template <int LT, bool FUSED, int TPB, bool OVERLAP = true, bool DET = false, bool STAMP = false, bool NOFLUSH = false>
__global__ void __launch_bounds__(TPB, (LT == 4 && TPB == 512) ? 2 : 4) msda_bwd_f32_tiled(
    const float* __restrict__ value, const float* __restrict__ loc, const float* __restrict__ attn, FrontEnd fe,
    const float* __restrict__ gout, TileGeom geo, int S, int M, float* __restrict__ gvalue,
    float* __restrict__ gloc, float* __restrict__ gattn, unsigned long long* __restrict__ gacc = nullptr,
    const unsigned* __restrict__ detscale = nullptr, unsigned long long* __restrict__ stamps = nullptr) {
  constexpr int D = 32, P = 4, LP = LT * P;
  constexpr int kBwdThreads = TPB, kBwdWaves = TPB / 64, kSortPerThread = kSortSamples / TPB;
  extern __shared__ __attribute__((aligned(16))) unsigned char lds_raw[];
  __shared__ TileState ts;
#define M2F_STAMP(k)                                                                                        \
  if constexpr (STAMP) {                                                                                    \
    if (threadIdx.x == 0)                                                                                   \
      stamps[static_cast<int64_t>(blockIdx.x) * 8 + (k)] = __builtin_amdgcn_s_memtime();                     \
  }

  // XCD-aware order: blocks are dealt round-robin over the 8 XCDs (b, b+8, ... share one); remap so each
  // XCD takes a contiguous run of (image, head) pairs, tile fastest, and its L2 holds one head's value
  // rows (2.75 MB per 1024^2 image) instead of several (speed only: any placement computes the same)
  const int ntiles = geo.nty * geo.ntx;
  const int nwg = gridDim.x, orig = blockIdx.x, xcd = orig & 7, q8 = nwg >> 3, r8 = nwg & 7;
  const int wg = (xcd < r8 ? xcd * (q8 + 1) : r8 * (q8 + 1) + (xcd - r8) * q8) + (orig >> 3);
  const int tile = wg % ntiles, pm = wg / ntiles, m = pm % M, n = pm / M;
  const int ty = tile / geo.ntx, tx = tile - ty * geo.ntx;
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int rs = M * D;  // value row stride (elements); N*S*M*D < 2^31 is checked on the host
  const int nsamp_max = geo.max_qt * LP;
  // LDS carve-up (16-byte aligned pieces): g rows [max_qt + 1][32] (the last a zero row: phase 3's padding records) |
  //   desc [max_qt * LP][4] | stage [waves][264] | cstart [max_cells + 1] i32 | oow [ceil(nsamp / 32)] u32
  //   | slots [max_qt * LP + 8] u32 | qmap [max_qt] i32
  float* gsh = reinterpret_cast<float*>(lds_raw);
  float* desc = gsh + (geo.max_qt + 1) * D;
  float* stage = desc + nsamp_max * 4;
  int* cstart = reinterpret_cast<int*>(stage + kBwdWaves * kStageFloats);
  unsigned* oow = reinterpret_cast<unsigned*>(cstart + ((geo.max_rows + 1 + 3) & ~3));
  unsigned* slots = reinterpret_cast<unsigned*>(oow + (((nsamp_max + 31) / 32 + 3) & ~3));
  int* qmap = reinterpret_cast<int*>(slots + nsamp_max + 8);  // pyramid position of each tile query
  float fxscale = 0.f;  // DET: 2^k, grad_value contributions leave the workgroup as round(v * 2^k) in int64
  bool fixed = false;
  if constexpr (DET) {
    fixed = detscale[1] == 0u;
    fxscale = det_scale(detscale[0], S);
  }
  // a grad_value contribution leaving the workgroup
  // (DET: a non-finite contribution -- a NaN / Inf from the projection's offsets or logits, which the pre-pass over
  // grad_output does not see -- goes to grad_value itself in fp32, where the conversion pass adds the fixed-point
  // sum to it: the element is then non-finite as the reference's atomics leave it)
  auto gv_add = [&](float* dst, float v) {
    if constexpr (DET) {
      if (fixed && __builtin_isfinite(v)) {
        atomicAdd(gacc + (dst - gvalue), static_cast<unsigned long long>(__float2ll_rn(v * fxscale)));
        return;
      }
    }
    atomicAdd(dst, v);
  };

  M2F_STAMP(5)
  if (tid < LT) {
    const int l = tid;
    const int y0 = tile_lo(ty, geo.H[l], geo.nty), y1 = tile_lo(ty + 1, geo.H[l], geo.nty);
    const int x0 = tile_lo(tx, geo.W[l], geo.ntx), x1 = tile_lo(tx + 1, geo.W[l], geo.ntx);
    ts.qy0[l] = y0;
    ts.qx0[l] = x0;
    ts.qw[l] = x1 - x0;
    ts.qc[l + 1] = (y1 - y0) * (x1 - x0);
    ts.bb[l][0] = 0x7fffffff; ts.bb[l][1] = -1; ts.bb[l][2] = 0x7fffffff; ts.bb[l][3] = -1;
    ts.H[l] = geo.H[l]; ts.W[l] = geo.W[l]; ts.start[l] = geo.start[l];
    ts.invW[l] = geo.invW[l]; ts.invH[l] = geo.invH[l];
  }
  for (int i = tid; i < (nsamp_max + 31) / 32; i += blockDim.x) oow[i] = 0u;
  for (int i = tid; i <= geo.max_rows; i += blockDim.x) cstart[i] = 0;  // the sort's counters (any window fits)
  if (tid == 0) ts.next_batch = kBwdWaves;
  if (tid < 64) ts.rbin[tid] = 0;
  if (tid < D) gsh[geo.max_qt * D + tid] = 0.f;   // the zero g row
  __syncthreads();
  if (tid == 0) {
    ts.qc[0] = 0;
    for (int l = 0; l < LT; ++l) ts.qc[l + 1] += ts.qc[l];
  }
  __syncthreads();
  const int Qt = ts.qc[LT];
  const int nsamp = Qt * LP;
  for (int qi = tid; qi < Qt; qi += blockDim.x) qmap[qi] = tile_query(ts, qi);
  __syncthreads();
  M2F_STAMP(0)

  // ---- phase 0: this head's grad_output rows of the tile's queries -> LDS (float4 per lane); the sample
  // descriptors (one lane per (query, level)) and the touched-corner boxes.  Every global load of the phase is
  // issued before any of its math or LDS stores (the g rows, then both task rounds' projection rows), so the
  // phase waits out one memory round trip instead of three ---------------------------------------------------
  constexpr int kGPre = 3;  // max_qt * 8 <= 3 * TPB at the default geometries; the rest loops
  f4 gpre[kGPre];
#pragma unroll
  for (int u = 0; u < kGPre; ++u) {
    const int idx = min(tid + u * kBwdThreads, Qt * 8 - 1), qi = idx >> 3, j = idx & 7;
    const int64_t pair = (static_cast<int64_t>(n) * S + qmap[qi]) * M + m;
    gpre[u] = ld4(gout + pair * D + 4 * j);
  }
  {
    int bmin_y[LT], bmax_y[LT], bmin_x[LT], bmax_x[LT];
#pragma unroll
    for (int l = 0; l < LT; ++l) { bmin_y[l] = 0x7fffffff; bmax_y[l] = -1; bmin_x[l] = 0x7fffffff; bmax_x[l] = -1; }
    // FUSED: a quad of lanes per query (lane l < LT handles level l), so the softmax over the pair's L*P
    // logits is shared: each lane exps its level's P logits, the quad max is a DPP reduction (exact), and
    // the sum is carried from lane to lane in logit order (the sequential sum the forward forms)
    // a quad of lanes per query either way (the op-level path with LT lanes per query ran 3-4 % slower: its
    // queries straddled quads and the level boxes took LT full-wave reductions)
    constexpr int TPQ = 4;  // tasks per query
    static_assert(LT <= 4, "one quad lane per level");
    const int ntask = Qt * TPQ;
    struct TaskIn {
      float x[P];      // logits (FUSED) or attention weights
      float2 xy[P];    // offsets (FUSED) or sampling locations
      float2 rf;       // reference point (FUSED)
    };
    auto task_load = [&](int t) {
      TaskIn in;
      t = min(t, ntask - 1);  // a spare round's addresses stay in range (its results are dropped)
      const int qi = t / TPQ, lt = t - qi * TPQ;
      const int l = lt < LT ? lt : LT - 1;
      const int64_t nq = static_cast<int64_t>(n) * S + qmap[qi];
      if constexpr (FUSED) {
        const float* prow = fe.proj + nq * fe.ld;
        const float* lg = prow + fe.lg0(m, M, LP) + l * P;
        const float* of = prow + fe.off0(m, LP) + l * P * 2;
#pragma unroll
        for (int p = 0; p < P; ++p) { in.x[p] = lg[p]; in.xy[p] = *reinterpret_cast<const float2*>(of + 2 * p); }
        in.rf = *reinterpret_cast<const float2*>(fe.ref + n * fe.ref_bs + (static_cast<int64_t>(qmap[qi]) * LT + l) * 2);
      } else {
        const int64_t kb = (nq * M + m) * LP + l * P;
#pragma unroll
        for (int p = 0; p < P; ++p) { in.xy[p] = *reinterpret_cast<const float2*>(loc + 2 * (kb + p)); in.x[p] = attn[kb + p]; }
        in.rf = make_float2(0.f, 0.f);
      }
      return in;
    };
    auto task_run = [&](int t, TaskIn& in) {  // whole quads run it together
      const int qi = t / TPQ, lt = t - qi * TPQ;
      const bool act = lt < LT;
      const int l = act ? lt : LT - 1;  // a spare quad lane mirrors the last level (its results are dropped)
      const int H = ts.H[l], W = ts.W[l];
      float av[P], lx[P], ly[P];
      if constexpr (FUSED) {
        float* x = in.x;
        float mx = -INFINITY;
#pragma unroll
        for (int p = 0; p < P; ++p) mx = fmaxf(mx, x[p]);
        mx = fmaxf(mx, qperm<0xB1>(mx));  // quad lanes 1 0 3 2
        mx = fmaxf(mx, qperm<0x4E>(mx));  // quad lanes 2 3 0 1
#pragma unroll
        for (int p = 0; p < P; ++p) x[p] = expf(x[p] - mx);
        float run = 0.f;
#pragma unroll
        for (int ll = 0; ll < LT; ++ll) {
          float prev = 0.f;
          if (ll > 0) {
            switch (ll) {  // broadcast quad lane ll - 1 (the DPP control must be an immediate)
              case 1: prev = qperm<0x00>(run); break;
              case 2: prev = qperm<0x55>(run); break;
              default: prev = qperm<0xAA>(run); break;
            }
          }
          if (lt == ll) {
            run = prev;
#pragma unroll
            for (int p = 0; p < P; ++p) run += x[p];
          }
        }
        float sum;
        switch (LT) {
          case 1: sum = qperm<0x00>(run); break;
          case 2: sum = qperm<0x55>(run); break;
          case 3: sum = qperm<0xAA>(run); break;
          default: sum = qperm<0xFF>(run); break;
        }
        const float inv = 1.f / sum;
        const float fW = static_cast<float>(W), fH = static_cast<float>(H);
        const float iW = ts.invW[l], iH = ts.invH[l];
        auto points = [&](auto pow2) {  // as msda_fused_fwd: exact reciprocals when W and H are powers of two
          constexpr bool POW2 = decltype(pow2)::value;
#pragma unroll
          for (int p = 0; p < P; ++p) {
            lx[p] = in.rf.x + div_norm(in.xy[p].x, fW, iW, POW2);
            ly[p] = in.rf.y + div_norm(in.xy[p].y, fH, iH, POW2);
            av[p] = x[p] * inv;
          }
        };
        if (((W & (W - 1)) | (H & (H - 1))) == 0) points(std::true_type{});
        else points(std::false_type{});
      } else {
#pragma unroll
        for (int p = 0; p < P; ++p) { lx[p] = in.xy[p].x; ly[p] = in.xy[p].y; av[p] = in.x[p]; }
      }
      if (!act) return;
      float* dq = desc + (qi * LP + l * P) * 4;
#pragma unroll
      for (int p = 0; p < P; ++p) {
        float h = ly[p] * H - 0.5f, w = lx[p] * W - 0.5f;
        const bool ok = h > -1.f && w > -1.f && h < static_cast<float>(H) && w < static_cast<float>(W);
        h = ok ? h : -2.f;
        w = ok ? w : -2.f;
        const float fh = floorf(h), fw = floorf(w);
        const int h0 = static_cast<int>(fh), w0 = static_cast<int>(fw);
        *reinterpret_cast<f4*>(dq + 4 * p) =
            f4{h - fh, w - fw, av[p], __uint_as_float(static_cast<unsigned>(h0 + 2) | (static_cast<unsigned>(w0 + 2) << 16))};
        if (ok) {
#pragma unroll
          for (int ll = 0; ll < LT; ++ll)
            if (ll == l) {
              bmin_y[ll] = min(bmin_y[ll], max(h0, 0)); bmax_y[ll] = max(bmax_y[ll], min(h0 + 1, H - 1));
              bmin_x[ll] = min(bmin_x[ll], max(w0, 0)); bmax_x[ll] = max(bmax_x[ll], min(w0 + 1, W - 1));
            }
        }
      }
    };
    // task rounds in pairs, both rounds' loads first (whole quads enter and leave together: ntask and the
    // round stride are multiples of 4)
    for (int t = tid; t < ntask; t += 2 * kBwdThreads) {
      TaskIn i0 = task_load(t), i1 = task_load(t + kBwdThreads);
      task_run(t, i0);
      if (t + kBwdThreads < ntask) task_run(t + kBwdThreads, i1);
    }
    // the g rows -> LDS (their loads were issued first)
#pragma unroll
    for (int u = 0; u < kGPre; ++u) {
      const int idx = tid + u * kBwdThreads;
      if (idx < Qt * 8) *reinterpret_cast<f4*>(gsh + g_chunk_off(idx >> 3, idx & 7)) = gpre[u];
    }
    for (int idx = tid + kGPre * kBwdThreads; idx < Qt * 8; idx += kBwdThreads) {
      const int qi = idx >> 3, j = idx & 7;
      const int64_t pair = (static_cast<int64_t>(n) * S + qmap[qi]) * M + m;
      *reinterpret_cast<f4*>(gsh + g_chunk_off(qi, j)) = ld4(gout + pair * D + 4 * j);
    }
    // per-level boxes over the wave, then over the workgroup
    {
      // a lane only ever touches its own level (tid & 3: the task stride is a multiple of 4), so the lanes of
      // one level (lane & 3 equal) reduce it over xor 4..32, and lane l < LT publishes level l
      const int ol = (lane & 3) < LT ? (lane & 3) : LT - 1;
      int a0 = 0x7fffffff, a1 = -1, a2 = 0x7fffffff, a3 = -1;
#pragma unroll
      for (int l = 0; l < LT; ++l)
        if (l == ol) { a0 = bmin_y[l]; a1 = bmax_y[l]; a2 = bmin_x[l]; a3 = bmax_x[l]; }
#pragma unroll
      for (int o = 32; o >= 4; o >>= 1) {
        a0 = min(a0, __shfl_xor(a0, o)); a1 = max(a1, __shfl_xor(a1, o));
        a2 = min(a2, __shfl_xor(a2, o)); a3 = max(a3, __shfl_xor(a3, o));
      }
      if (lane < LT && a1 >= 0) {
        atomicMin(&ts.bb[lane][0], a0); atomicMax(&ts.bb[lane][1], a1);
        atomicMin(&ts.bb[lane][2], a2); atomicMax(&ts.bb[lane][3], a3);
      }
    }
  }
  __syncthreads();
  M2F_STAMP(1)

  // ---- window: touched box clipped to the tile +- halo; the halo shrinks until the cells fit ----------
  if (tid == 0) {
    for (int halo = geo.max_halo; halo >= 0; --halo) {
      int rows = 0, cells = 0;
      for (int l = 0; l < LT; ++l) {
        const int H = geo.H[l], W = geo.W[l];
        const int ry0 = max(tile_lo(ty, H, geo.nty) - halo, 0), ry1 = min(tile_lo(ty + 1, H, geo.nty) - 1 + halo, H - 1);
        const int rx0 = max(tile_lo(tx, W, geo.ntx) - halo, 0), rx1 = min(tile_lo(tx + 1, W, geo.ntx) - 1 + halo, W - 1);
        const int wy0 = max(ry0, ts.bb[l][0]), wy1 = min(ry1, ts.bb[l][1]);
        const int wx0 = max(rx0, ts.bb[l][2]), wx1 = min(rx1, ts.bb[l][3]);
        const bool any = wy1 >= wy0 && wx1 >= wx0;
        ts.wy0[l] = wy0; ts.wx0[l] = wx0;
        ts.wh[l] = any ? wy1 - wy0 + 1 : 0; ts.ww[l] = any ? wx1 - wx0 + 1 : 0;
        ts.iww[l] = any ? 1.f / static_cast<float>(ts.ww[l]) : 0.f;
        ts.roff[l] = rows;
        ts.coff[l] = cells;
        rows += ts.wh[l] * ts.ww[l];
        cells += any ? (ts.wh[l] + 1) * (ts.ww[l] + 1) : 0;
      }
      ts.roff[LT] = rows;
      ts.coff[LT] = cells;
      if (cells <= geo.max_rows) break;
      if (halo == 0) {  // cannot happen when the budget covers a tile's own footprint; stay correct anyway
        for (int l = 0; l <= LT; ++l) { ts.roff[l] = 0; ts.coff[l] = 0; }
        for (int l = 0; l < LT; ++l) { ts.wh[l] = 0; ts.ww[l] = 0; }
      }
    }
  }
  __syncthreads();
  const int cells_total = ts.coff[LT];

  // ---- phase 1: counting sort of the in-window samples by cell ------------------------------------------
  {
    int cell[kSortPerThread], rank[kSortPerThread];
#pragma unroll
    for (int r = 0; r < kSortPerThread; ++r) {
      const int sid = tid + r * kBwdThreads;
      cell[r] = -1;
      if (sid < nsamp) {
        const unsigned pk = __float_as_uint(desc[4 * sid + 3]);
        const int h0 = static_cast<int>(pk & 0xffffu) - 2, w0 = static_cast<int>(pk >> 16) - 2;
        if (h0 != -2) {  // ok sample
          const int l = (sid % LP) / P;
          const int c = window_cell(ts, l, h0, w0, ts.H[l], ts.W[l]);
          if (c >= 0) {
            cell[r] = c;
            rank[r] = atomicAdd(cstart + c, 1);
          } else {
            atomicOr(oow + (sid >> 5), 1u << (sid & 31));
          }
        }
      }
    }
    __syncthreads();
    // exclusive scan of cstart[0 .. cells_total] (cstart[cells_total] = 0 -> total)
    const int per = (cells_total + 1 + kBwdThreads - 1) / kBwdThreads;
    const int c0 = tid * per;
    int run = 0;
    for (int i = 0; i < per; ++i) run += (c0 + i <= cells_total) ? cstart[c0 + i] : 0;
    const int incl = wave_incl_scan(run, lane);
    if (lane == 63) ts.wsum[wid] = incl;
    __syncthreads();
    int wbase = 0;
    for (int w = 0; w < wid; ++w) wbase += ts.wsum[w];
    int acc = wbase + incl - run;
    for (int i = 0; i < per; ++i) {
      if (c0 + i <= cells_total) {
        const int v = cstart[c0 + i];
        cstart[c0 + i] = acc;
        acc += v;
      }
    }
    __syncthreads();
#pragma unroll
    for (int r = 0; r < kSortPerThread; ++r)
      if (cell[r] >= 0) {  // slot = sample index << 16 | g row byte offset: phase 3 decodes it in 3 VALU
        const int sid = tid + r * kBwdThreads, qs = sid / LP;
        slots[cstart[cell[r]] + rank[r]] =
            (static_cast<unsigned>(sid) << 16) | static_cast<unsigned>(4 * g_chunk_off(qs, 0));
      }
  }
  __syncthreads();
  if constexpr (DET) {
    // a cell's slots in sample order (the ranks above come from LDS atomics, in arrival order): insertion sort,
    // one thread per cell (a cell holds a few samples)
    for (int c = tid; c < cells_total; c += kBwdThreads) {
      const int b0 = cstart[c], b1 = cstart[c + 1];
      for (int i = b0 + 1; i < b1; ++i) {
        const unsigned key = slots[i];
        int k = i - 1;
        while (k >= b0 && slots[k] > key) { slots[k + 1] = slots[k]; --k; }
        slots[k + 1] = key;
      }
    }
    __syncthreads();
  }
  // ---- phase-3 rows in order of their record count, heaviest first -------------------------------------------------
  // A phase-3 unit is 16 rows walked in lockstep by the wave's 4-lane groups, so it takes as long as its longest list;
  // in window order neighbouring rows' lists differ several-fold (the lists of a 16-row unit averaged 0.43 of its
  // longest at config 2 near-init, a host count).  A counting sort over 64 bins of 4 records each deals units of rows
  // with lists of nearly equal length.  The permutation lives in the high halves of cstart's words (every cstart value
  // is < 2^16; rows_total <= cells_total), read by phase 3 with 16-bit loads; a window too large for the per-thread
  // row registers keeps window order.
  constexpr int kRowsPT = 4, kRowBins = 64, kRowBinShift = 2;
  const int rows_all = ts.roff[LT];
  const bool rowsort = geo.rowsort != 0 && rows_all <= kRowsPT * kBwdThreads;
  // window row -> (level, window y, window x, its cell index, the cell grid width)
  auto row_cell = [&](int row, int& l, int& ey, int& ex, int& cbase, int& cw) {
    l = 0;
    while (row >= ts.roff[l + 1]) ++l;
    const int ww = ts.ww[l], rr = row - ts.roff[l];
    // rr / ww by the reciprocal: (rr + 0.5) / ww is at least 0.5 / ww from an integer and the product's error
    // is below wh * ww * 2^-23 / ww, so the truncation is exact for windows of fewer than 2^22 cells
    ey = static_cast<int>((static_cast<float>(rr) + 0.5f) * ts.iww[l]);
    ex = rr - ey * ww;  // window coordinates; cells are offset by (1, 1)
    cw = ww + 1;
    cbase = ts.coff[l] + (ey + 1) * cw + ex + 1;
  };
  const unsigned short* cs16 = reinterpret_cast<const unsigned short*>(cstart);   // the cstart values (low halves)
  if (rowsort) {
    int rk[kRowsPT], bk[kRowsPT];
#pragma unroll
    for (int i = 0; i < kRowsPT; ++i) {
      const int row = tid + i * kBwdThreads;
      bk[i] = -1;
      if (row < rows_all) {
        int l, ey, ex, cbase, cw;
        row_cell(row, l, ey, ex, cbase, cw);
        const int n = (cstart[cbase + 1] - cstart[cbase - 1]) + (cstart[cbase - cw + 1] - cstart[cbase - cw - 1]);
        bk[i] = kRowBins - 1 - min(n >> kRowBinShift, kRowBins - 1);
        rk[i] = atomicAdd(&ts.rbin[bk[i]], 1);
      }
    }
    __syncthreads();
    if (wid == 0) {   // exclusive scan of the 64 bins
      const int v = ts.rbin[lane];
      ts.rbin[lane] = wave_incl_scan(v, lane) - v;
    }
    __syncthreads();
    unsigned short* hi16 = reinterpret_cast<unsigned short*>(cstart);
#pragma unroll
    for (int i = 0; i < kRowsPT; ++i)
      if (bk[i] >= 0) hi16[2 * (ts.rbin[bk[i]] + rk[i]) + 1] = static_cast<unsigned short>(tid + i * kBwdThreads);
    __syncthreads();
  }
  M2F_STAMP(2)

  // ---- phases 2 and 3: one work queue ----------------------------------------------------------------------
  // Phase 2 (16 queries per unit) gathers the samples' corner rows through L1 (texture-path bound); phase 3 (16
  // window rows per unit) walks the slot lists in LDS (LDS bound).  Neither reads what the other writes (phase 3
  // derives its corner coefficients from the {h, w, a} descriptors), so with OVERLAP the units of both kinds are
  // dealt from one LDS counter, interleaved, and the waves of a workgroup run both at once instead of one phase
  // after a barrier.
  {
    const int rows_total = ts.roff[LT];
    constexpr int LPR = kWalkLanes, CPL = D / LPR, RPW = 64 / LPR;  // phase 3: lanes per row, channels per lane, rows per wave
    const int U2 = (Qt + 15) / 16, U3 = (rows_total + RPW - 1) / RPW;
    const int ratio = max(geo.ratio23, 1);
    // phase 2, quad form: a quad of lanes takes one query, lane j owning channels 4j..4j+3 and 16+4j..16+4j+3
    // (one load address per corner row: the second half is the immediate offset).  Per level, lane j derives
    // point j's geometry once; the quad takes the points in turn with the owner's corner byte offsets by DPP
    // broadcast, each lane forming 16 partial channel dots (4 points x 4 corners) over its 8 channels; a two-stage
    // quad transpose-reduce (xor 2, xor 1) leaves lane j the 4 full corner dots of ITS point, so the gradient math
    // and the stores run once per point.
    const int j = lane & 3, gq = lane >> 2;
    const unsigned cjb = 16u * j;
    const char* vbytes = reinterpret_cast<const char*>(value);
    char* gvbytes = reinterpret_cast<char*>(gvalue);
    const int rsb = rs * 4;  // value row stride in bytes; value bytes < 2^31 (host check)
    auto phase2_unit = [&](int unit) {
      const int qi = unit * 16 + gq;
      if (qi >= Qt) return;  // whole quad (same qi) idles together
      const int q = qmap[qi];
      const int64_t nq = static_cast<int64_t>(n) * S + q;
      const f4 gA = *reinterpret_cast<const f4*>(gsh + g_chunk_off(qi, j));
      const f4 gB = *reinterpret_cast<const f4*>(gsh + g_chunk_off(qi, 4 + j));
      const float* dq = desc + qi * LP * 4;
      const int sid0 = qi * LP, sh = sid0 & 31;
      const unsigned w0f = oow[sid0 >> 5], w1f = oow[min((sid0 + LP - 1) >> 5, (nsamp_max + 31) / 32 - 1)];
      const unsigned qfar = (sh ? (w0f >> sh) | (w1f << (32 - sh)) : w0f) & ((1u << LP) - 1u);
      float dot = 0.f;  // FUSED: this lane's points' sum of a * d attn
      float gaown[LT], aown[LT];
#pragma unroll
      for (int l = 0; l < LT; ++l) {
        const int H = geo.H[l], W = geo.W[l];
        const int lbase = ((n * S + geo.start[l]) * M + m) * D * 4;
        // this lane's point (l, j)
        const f4 dk = *reinterpret_cast<const f4*>(dq + 4 * (l * P + j));
        const float a = dk[2];
        // not-ok samples carry floors -2 (every corner outside, ok false)
        const unsigned pk = __float_as_uint(dk[3]);
        const QuadPoint k = quad_point_fl(static_cast<int>(pk & 0xffffu) - 2, static_cast<int>(pk >> 16) - 2, dk[0], dk[1],
                                          H, W, lbase, rsb);
        const bool ok = k.ok;
        const float ly = k.ly, lx = k.lx, hy = 1.f - ly, hx = 1.f - lx;
        const int o1 = k.o1, o2 = k.o2, o3 = k.o3, o4 = k.o4;
        // partial channel dots over this lane's 8 channels, pairs of channels in packed fp32 FMAs (v_pk_fma_f32)
        auto dot8 = [&](const f4& va, const f4& vb) {
          f2 t = f2{va.x, va.y} * f2{gA.x, gA.y};
          t = __builtin_elementwise_fma(f2{va.z, va.w}, f2{gA.z, gA.w}, t);
          t = __builtin_elementwise_fma(f2{vb.x, vb.y}, f2{gB.x, gB.y}, t);
          t = __builtin_elementwise_fma(f2{vb.z, vb.w}, f2{gB.z, gB.w}, t);
          return t.x + t.y;
        };
        const bool hi2 = (j & 2) != 0, hi1 = (j & 1) != 0;
        float s1[2][4];
        // one point at a time (8 corner loads in flight per lane: the texture path, not latency, bounds this phase,
        // and fewer registers keep the merged phase 2/3 loop free of spills); after the points {0, 2} and {1, 3} the
        // first transpose-reduce stage (xor 2) folds their 8 partial dots to 4: lanes {0, 1} keep the lower point,
        // lanes {2, 3} the upper one, summed over the lane pair
        auto point_dots = [&](auto cc, float* part) {
          constexpr int C = decltype(cc)::value;
          const char* vhi = vbytes + 64;  // the row's second half: an immediate offset
          const unsigned b1 = qpermi<C>(o1) + cjb, b2 = qpermi<C>(o2) + cjb;
          const unsigned b3 = qpermi<C>(o3) + cjb, b4 = qpermi<C>(o4) + cjb;
          const f4 v0 = ldb4(vbytes, b1), v1 = ldb4(vhi, b1), v2 = ldb4(vbytes, b2), v3 = ldb4(vhi, b2);
          const f4 v4 = ldb4(vbytes, b3), v5 = ldb4(vhi, b3), v6 = ldb4(vbytes, b4), v7 = ldb4(vhi, b4);
          part[0] = dot8(v0, v1);
          part[1] = dot8(v2, v3);
          part[2] = dot8(v4, v5);
          part[3] = dot8(v6, v7);
        };
        auto stage1 = [&](const float* plo, const float* phi, float* out) {
#pragma unroll
          for (int c = 0; c < 4; ++c) {
            const float lo = plo[c] + qpermf<0x4E>(plo[c]), hi = phi[c] + qpermf<0x4E>(phi[c]);
            out[c] = hi2 ? hi : lo;
          }
        };
        {
          float pa_[4], pb_[4];
          point_dots(std::integral_constant<int, 0x00>{}, pa_);
          point_dots(std::integral_constant<int, 0xAA>{}, pb_);
          stage1(pa_, pb_, s1[0]);
          point_dots(std::integral_constant<int, 0x55>{}, pa_);
          point_dots(std::integral_constant<int, 0xFF>{}, pb_);
          stage1(pa_, pb_, s1[1]);
        }
        // second stage (xor 1): lane j holds the full corner dots of point j
        float dd[4];
#pragma unroll
        for (int c = 0; c < 4; ++c) {
          const float lo = s1[0][c] + qpermf<0xB1>(s1[0][c]);
          const float hi = s1[1][c] + qpermf<0xB1>(s1[1][c]);
          dd[c] = hi1 ? hi : lo;
        }
        // a corner outside the level contributes nothing (as the reference, which skips it)
        const float d1 = k.c1 ? dd[0] : 0.f, d2 = k.c2 ? dd[1] : 0.f, d3 = k.c3 ? dd[2] : 0.f, d4 = k.c4 ? dd[3] : 0.f;
        const float pa = k.w1 * d1 + k.w2 * d2 + k.w3 * d3 + k.w4 * d4;
        const float px = a * (hy * (d2 - d1) + ly * (d4 - d3));
        const float py = a * (hx * (d3 - d1) + lx * (d4 - d2));
        if constexpr (FUSED) {
          const float gak = ok ? pa : 0.f;
          dot = fmaf(a, gak, dot);
          gaown[l] = gak;
          aown[l] = a;
          *reinterpret_cast<float2*>(gloc + nq * (3 * M * LP) + fe.off0(m, LP) + l * P * 2 + 2 * j) =
              ok ? make_float2(px, py) : make_float2(0.f, 0.f);
        } else {
          const unsigned kl = ((static_cast<unsigned>(n * S + q) * M + m) * LT + l) * P + j;  // < 2^28 (host)
          *reinterpret_cast<float*>(reinterpret_cast<char*>(gattn) + kl * 4u) = ok ? pa : 0.f;
          *reinterpret_cast<float2*>(reinterpret_cast<char*>(gloc) + kl * 8u) =
              ok ? make_float2(W * px, H * py) : make_float2(0.f, 0.f);
        }
        // out-of-window points (rare; flags are per query, so quad-uniform): every lane adds its 8 channels of
        // the point's 4 corner rows straight to HBM (fp32 atomics, as the reference)
        if ((qfar >> (l * P)) & 0xFu) {
          const int cf = (k.c1 ? 1 : 0) | (k.c2 ? 2 : 0) | (k.c3 ? 4 : 0) | (k.c4 ? 8 : 0);
          const float wt1 = k.w1 * a, wt2 = k.w2 * a, wt3 = k.w3 * a, wt4 = k.w4 * a;
          auto scatter = [&](auto cc, int p) {
            constexpr int C = decltype(cc)::value;
            const int f = qpermi<C>(cf);
            const unsigned b1 = qpermi<C>(o1) + cjb, b2 = qpermi<C>(o2) + cjb;
            const unsigned b3 = qpermi<C>(o3) + cjb, b4 = qpermi<C>(o4) + cjb;
            const float u1 = qpermf<C>(wt1), u2 = qpermf<C>(wt2), u3 = qpermf<C>(wt3), u4 = qpermf<C>(wt4);
            if ((qfar >> (l * P + p)) & 1u) {
              auto add8 = [&](unsigned boff, float u) {
                float* o = reinterpret_cast<float*>(gvbytes + boff);
                const f4 ta = u * gA, tb = u * gB;
                gv_add(o, ta.x); gv_add(o + 1, ta.y); gv_add(o + 2, ta.z); gv_add(o + 3, ta.w);
                gv_add(o + 16, tb.x); gv_add(o + 17, tb.y); gv_add(o + 18, tb.z); gv_add(o + 19, tb.w);
              };
              if (f & 1) add8(b1, u1);
              if (f & 2) add8(b2, u2);
              if (f & 4) add8(b3, u3);
              if (f & 8) add8(b4, u4);
            }
          };
          scatter(std::integral_constant<int, 0x00>{}, 0);
          scatter(std::integral_constant<int, 0x55>{}, 1);
          scatter(std::integral_constant<int, 0xAA>{}, 2);
          scatter(std::integral_constant<int, 0xFF>{}, 3);
        }
      }
      if constexpr (FUSED) {
        // softmax backward over the pair's L*P logits: d logit_k = a_k (d a_k - sum_i a_i d a_i)
        dot += qpermf<0xB1>(dot);
        dot += qpermf<0x4E>(dot);
        float* gl = gloc + nq * (3 * M * LP) + fe.lg0(m, M, LP);
#pragma unroll
        for (int l = 0; l < LT; ++l) gl[l * P + j] = aown[l] * (gaown[l] - dot);
      }
    };
    // phase 3: per window pixel, the 4 covering slot ranges; one row-contiguous atomic add per row
    const int jl = lane % LPR, rw = lane / LPR;
    float* wst = stage + wid * kStageFloats;               // this wave's flush half: 8 rows x 32 channels
    int* woff = reinterpret_cast<int*>(wst + 8 * 32);      // and their grad_value element offsets
    const char* gbytes = reinterpret_cast<const char*>(gsh);
    const unsigned jlb = static_cast<unsigned>(CPL * 4 * jl);  // this lane's channel bytes (< 128: ORs into a row offset)
    auto phase3_unit = [&](int unit) {
      const int base = unit * RPW;
      int row = base + rw;
      if (rowsort && row < rows_total) row = cs16[2 * row + 1];   // the row sort's permutation
      float acc[CPL];
#pragma unroll
      for (int k = 0; k < CPL; ++k) acc[k] = 0.f;
      int off = -1;  // element offset of channel 0 of this group's grad_value row (-1: none)
      int l = 0, ey = 0, ex = 0;
      bool any = false;
      if (row < rows_total) {
        int cbase, cw;
        row_cell(row, l, ey, ex, cbase, cw);
        // corner 1 of cell (y, x), corner 2 of (y, x-1), corner 3 of (y-1, x), corner 4 of (y-1, x-1).  Cells are
        // numbered row-major, so the slot ranges of (y, x-1) and (y, x) are one contiguous range, as are those of
        // (y-1, x-1) and (y-1, x): two walks, the six range bounds read up front (16-bit reads: the high halves
        // may hold the row sort's permutation)
        const unsigned short* cs = cs16 + 2 * cbase;
        const int b0 = cs[-2], b1 = cs[0], b2 = cs[2];
        const int u0 = cs[-2 * cw - 2], u1 = cs[-2 * cw], u2 = cs[-2 * cw + 2];
        any = b2 > b0 || u2 > u0;
        // HI: the row above (corners 3 / 4: ly a, else (1 - ly) a); a record below `mid` comes from the cell at x-1
        // (corners 2 / 4: times lx, else (1 - lx)); the (1 - t) factors as fmas
        auto walk = [&](auto hi_c, int s0, int mid, int s1) {
          constexpr bool HI = decltype(hi_c)::value;
          // a record: the sample's descriptor {ly, lx, a, -} (one 16-byte read) and its query's g row
          auto rec = [&](unsigned p, int idx) {
            const f4 dk = *reinterpret_cast<const f4*>(reinterpret_cast<const char*>(desc) + ((p >> 12) & 0xffff0u));
            const float ly = dk[0], lx = dk[1], a = dk[2];
            const float A = HI ? ly * a : fmaf(-ly, a, a);
            const f4* g = reinterpret_cast<const f4*>(gbytes + ((p & 0xffffu) | jlb));
            const float cf = idx < mid ? A * lx : fmaf(-A, lx, A);
#pragma unroll
            for (int k = 0; k < CPL / 4; ++k) {  // fma chains (pairs of channels pack into v_pk_fma_f32)
              const f4 v = g[k];
#pragma unroll
              for (int e = 0; e < 4; ++e) acc[4 * k + e] = fmaf(cf, v[e], acc[4 * k + e]);
            }
          };
          // two records per step, the next pair's slots read one step ahead (unclamped: a read past the range, or
          // past the array into its 8-entry pad, is never used), so a step waits on one LDS round trip
          const unsigned* sp = slots + s0;
          unsigned npa = sp[0], npb = sp[1];
          int i = s0;
          for (; i + 1 < s1; i += 2, sp += 2) {
            const unsigned pa = npa, pb = npb;
            npa = sp[2];
            npb = sp[3];
            rec(pa, i);
            rec(pb, i + 1);
          }
          if (i < s1) rec(npa, i);
        };
        // quad form (msda_bwd_walk4, the default): four records per step, lane jl of the row's quad decoding record
        // i + jl once (slot, descriptor, coefficient) and the quad taking the four in turn with the coefficient and
        // the g-row offset broadcast by DPP (the broadcast folds into the FMAs / the address add): per record 1 + 8
        // VALU per lane instead of ~6 + 8 and a quarter of the descriptor reads; a range's tail records carry
        // coefficient 0 (any in-range slot read: the 8-entry pad covers the read past the range)
        auto walk4 = [&](auto hi_c, int s0, int mid, int s1) {
          constexpr bool HI = decltype(hi_c)::value;
          unsigned np = slots[s0 + jl];
          for (int i = s0; i < s1; i += 4) {
            const int idx = i + jl;
            // a padding record: descriptor 0, the zero g row (coefficient 0 times zeros: nothing added, whatever
            // non-finite values other g rows hold)
            const unsigned p = idx < s1 ? np : static_cast<unsigned>(geo.max_qt * D * 4);
            np = slots[idx + 4];
            const f4 dk = *reinterpret_cast<const f4*>(reinterpret_cast<const char*>(desc) + ((p >> 12) & 0xffff0u));
            const float ly = dk[0], lx = dk[1], a = dk[2];
            const float A = HI ? ly * a : fmaf(-ly, a, a);
            float cf = idx < mid ? A * lx : fmaf(-A, lx, A);
            cf = idx < s1 ? cf : 0.f;
            const unsigned gb = p & 0xffffu;
            auto rec4 = [&](auto cc) {
              constexpr int C = decltype(cc)::value;
              const float c = qpermf<C>(cf);
              const f4* g = reinterpret_cast<const f4*>(gbytes + (static_cast<unsigned>(qpermi<C>(static_cast<int>(gb))) | jlb));
#pragma unroll
              for (int k = 0; k < CPL / 4; ++k) {
                const f4 v = g[k];
#pragma unroll
                for (int e = 0; e < 4; ++e) acc[4 * k + e] = fmaf(c, v[e], acc[4 * k + e]);
              }
            };
            rec4(std::integral_constant<int, 0x00>{});
            rec4(std::integral_constant<int, 0x55>{});
            rec4(std::integral_constant<int, 0xAA>{});
            rec4(std::integral_constant<int, 0xFF>{});
          }
        };
        if (geo.walk4) {
          walk4(std::false_type{}, b0, b1, b2);
          walk4(std::true_type{}, u0, u1, u2);
        } else {
          walk(std::false_type{}, b0, b1, b2);
          walk(std::true_type{}, u0, u1, u2);
        }
      }
      if (any) {
        const int y = ts.wy0[l] + ey, x = ts.wx0[l] + ex;
        off = ((n * S + ts.start[l] + y * ts.W[l] + x) * M + m) * D;
      }
      // transpose the wave's RPW rows through LDS, 8 rows at a time, so that each atomic instruction adds two whole
      // 128-B rows, one dword per lane (the L2 takes atomics per 64-B request)
#pragma unroll
      for (int half = 0; half < RPW / 8; ++half) {
        if ((rw >> 3) == half) {
#pragma unroll
          for (int k = 0; k < CPL / 4; ++k)
            *reinterpret_cast<f4*>(wst + (rw & 7) * 32 + CPL * jl + 4 * k) =
                f4{acc[4 * k], acc[4 * k + 1], acc[4 * k + 2], acc[4 * k + 3]};
          if (jl == 0) woff[rw & 7] = off;
        }
        __builtin_amdgcn_s_waitcnt(0xC07F);  // lgkmcnt(0): this wave's stage writes are in LDS
        __builtin_amdgcn_wave_barrier();
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          const int r2 = 2 * i + (lane >> 5);
          const int o = woff[r2];
          const float v = wst[r2 * 32 + (lane & 31)];
          if constexpr (NOFLUSH) {
            asm volatile("" ::"v"(v), "v"(o));
          } else {
            if (o >= 0) gv_add(gvalue + o + (lane & 31), v);
          }
        }
        __builtin_amdgcn_s_waitcnt(0xC07F);  // reads done before the stage is written again
        __builtin_amdgcn_wave_barrier();
      }
    };
    auto next_unit = [&]() {
      int nb = 0;
      if (lane == 0) nb = atomicAdd(&ts.next_batch, 1);
      return __builtin_amdgcn_readlane(nb, 0);   // lane 0's value, uniform (not an LDS permute round trip)
    };
    if constexpr (OVERLAP) {
      // R phase-2 units per phase-3 unit while phase 2 lasts (msda_bwd_ratio, default 1), then the rest of phase 3:
      // with c3(k) = max(min(U3, k / (R + 1)), k - U2) phase-3 units among the first k, unit u is phase-3 unit c3(u)
      // when c3 steps up at u, else phase-2 unit u - c3(u).  Texture-path work early, LDS work to the end (a
      // schedule spreading the phase-2 units evenly over the queue measured 2.7 % slower: a gather unit late in
      // the queue is a straggler); the coarse levels' rows come first (~37 records each at config 2 against ~9)
      const int T = U2 + U3, R1 = ratio + 1;
      for (int u = wid; u < T; u = next_unit()) {
        const int c0 = max(min(U3, u / R1), u - U2), c1 = max(min(U3, (u + 1) / R1), u + 1 - U2);
        if (c1 > c0) phase3_unit(c0);
        else phase2_unit(u - c0);
      }
    } else {
      for (int u = wid; u < U2; u += kBwdWaves) phase2_unit(u);
      __syncthreads();
      M2F_STAMP(3)
      for (int u = wid; u < U3; u = next_unit()) phase3_unit(u);
    }
  }
  if constexpr (STAMP) __syncthreads();
  M2F_STAMP(4)
#undef M2F_STAMP
}

// ------------------------------------------------------------------------------------------------
// Fused front end, forward: the MSDA forward reading the raw projection (offsets | logits) and the
// reference points instead of materialised sampling_locations / attention_weights.  Per pair the 8-lane
// group computes softmax over the L*P logits and loc = ref + offset / (W_l, H_l) exactly as the
// reference module does (ms_deform_attn.py:102-109), then samples as msda_fwd_f32_vec.
// ------------------------------------------------------------------------------------------------
//
// TILED: a workgroup takes one head of an 8 x 4 patch of queries of one level instead of 4 consecutive
// queries x 8 heads, with the head as the fastest block index: every XCD (blocks are dealt round-robin)
// then gathers one head's value rows (2.75 MB per 1024^2 image, L2-resident) and a block's 32 queries
// sample one compact neighbourhood of them (L1 reuse across the patch).  Needs Lq == S (encoder queries
// are the pixels).
// OFF32: every element offset of value / out fits 32 bits (checked on the host): 32-bit corner addressing.
template <int LT, bool TILED, bool OFF32>
__global__ void __launch_bounds__(256) msda_fused_fwd(const float* __restrict__ value, FrontEnd fe, TileGeom geo,
                                                      int64_t npairs, int S, int M, int Lq, float* __restrict__ out) {
  constexpr int D = 32, G = 8, P = 4, LP = LT * P;
  int64_t pair, n;
  int m, q;
  if constexpr (TILED) {
    const int g = threadIdx.x / G;
    int64_t b = blockIdx.x;
    m = static_cast<int>(b % M);
    b /= M;
    int T = 0;
#pragma unroll
    for (int l = 0; l < LT; ++l) T += ((geo.H[l] + 3) / 4) * ((geo.W[l] + 7) / 8);
    n = b / T;
    int t = static_cast<int>(b - n * T);
    int lv = 0;
#pragma unroll
    for (int l = 0; l < LT - 1; ++l) {
      const int nt = ((geo.H[l] + 3) / 4) * ((geo.W[l] + 7) / 8);
      if (lv == l && t >= nt) { t -= nt; lv = l + 1; }
    }
    const int H = geo.H[lv], W = geo.W[lv], tlx = (W + 7) / 8;
    const int y = (t / tlx) * 4 + (g >> 3), x = (t % tlx) * 8 + (g & 7);
    if (y >= H || x >= W) return;
    q = geo.start[lv] + y * W + x;
    pair = (n * Lq + q) * M + m;
  } else {
    pair = static_cast<int64_t>(blockIdx.x) * (256 / G) + threadIdx.x / G;
    if (pair >= npairs) return;
    m = static_cast<int>(pair % M);
    const int64_t nq0 = pair / M;
    n = nq0 / Lq;
    q = static_cast<int>(nq0 - n * Lq);
  }
  const int j = threadIdx.x % G;
  const int64_t nq = n * Lq + q;
  const int64_t rs = static_cast<int64_t>(M) * D;
  const float* prow = fe.proj + nq * fe.ld;
  const float* rrow = fe.ref + n * fe.ref_bs + static_cast<int64_t>(q) * LT * 2;
  const float* lg = prow + fe.lg0(m, M, LP);
  // softmax over the pair's L*P logits (ms_deform_attn.py:103-104), each exp computed once in the group:
  // lane j owns logits j and j + 8, the group max is a DPP reduction (exact), and every lane gathers the
  // twelve exps and sums them in logit order (the backward recomputes the same sum, msda_bwd_f32_tiled)
  static_assert(LP <= 16, "two logits per lane of the 8-lane group");
  const float l0 = j < LP ? lg[j] : -INFINITY, l1 = j + 8 < LP ? lg[j + 8] : -INFINITY;
  const float mx = max8_dpp(fmaxf(l0, l1));
  const float e0 = j < LP ? expf(l0 - mx) : 0.f, e1 = j + 8 < LP ? expf(l1 - mx) : 0.f;
  const int gb = (threadIdx.x & 63) & ~(G - 1);
  float a[LP];
  float sum = 0.f;
#pragma unroll
  for (int k = 0; k < LP; ++k) {
    a[k] = __shfl(k < 8 ? e0 : e1, gb + (k & 7));
    sum += a[k];
  }
  const float inv = 1.f / sum;
  const f4 z = {0.f, 0.f, 0.f, 0.f};
  f4 acc = z;
#pragma unroll
  for (int l = 0; l < LT; ++l) {
    const int H = geo.H[l], W = geo.W[l];
    const int64_t lbase = ((n * S + geo.start[l]) * M + m) * D + 4 * j;
    const float2 rf = *reinterpret_cast<const float2*>(rrow + 2 * l);
    const float fW = static_cast<float>(W), fH = static_cast<float>(H);
    const float iW = 1.f / fW, iH = 1.f / fH;
    // the level's points; POW2 (W and H powers of two, wave-uniform): offsets scaled by the exact reciprocals
    auto points = [&](auto pow2) {
      constexpr bool POW2 = decltype(pow2)::value;
#pragma unroll
      for (int p = 0; p < P; ++p) {
        const float2 off = *reinterpret_cast<const float2*>(prow + fe.off0(m, LP) + (l * P + p) * 2);
        const float sx = rf.x + div_norm(off.x, fW, iW, POW2);
        const float sy = rf.y + div_norm(off.y, fH, iH, POW2);
        f4 val;
        bool ok;
        if constexpr (OFF32) {
          const Corners32 k = make_corners32(sx, sy, H, W, static_cast<int>(lbase), static_cast<int>(rs));
          const f4 v1 = ld4(value + k.o1), v2 = ld4(value + k.o2), v3 = ld4(value + k.o3), v4 = ld4(value + k.o4);
          // a corner outside the level of an in-range sample gets weight 0 instead of a zeroed row (one select,
          // not four): its clamped row is always another corner of the same sample, so the output is non-finite
          // in exactly the elements where the reference's is (only Inf may read as NaN); an out-of-range sample
          // (clamped onto the level's first pixel) is dropped by the select on its sum below
          const float w1 = k.c1 ? k.w1 : 0.f, w2 = k.c2 ? k.w2 : 0.f, w3 = k.c3 ? k.w3 : 0.f, w4 = k.c4 ? k.w4 : 0.f;
          val = w1 * v1 + w2 * v2 + w3 * v3 + w4 * v4;
          ok = k.ok;
        } else {
          const Corners k = make_corners(sx, sy, H, W, lbase, rs);
          f4 v1 = ld4(value + k.o1), v2 = ld4(value + k.o2), v3 = ld4(value + k.o3), v4 = ld4(value + k.o4);
          v1 = k.c1 ? v1 : z; v2 = k.c2 ? v2 : z; v3 = k.c3 ? v3 : z; v4 = k.c4 ? v4 : z;
          val = k.w1 * v1 + k.w2 * v2 + k.w3 * v3 + k.w4 * v4;
          ok = k.ok;
        }
        // a not-ok sample is dropped by one select on its sum, then one fma per channel
        const float wa = a[l * P + p] * inv;
        val = ok ? val : z;
        acc.x = fmaf(val.x, wa, acc.x); acc.y = fmaf(val.y, wa, acc.y);
        acc.z = fmaf(val.z, wa, acc.z); acc.w = fmaf(val.w, wa, acc.w);
      }
    };
    if (((W & (W - 1)) | (H & (H - 1))) == 0) points(std::true_type{});
    else points(std::false_type{});
  }
  *reinterpret_cast<f4*>(out + pair * D + 4 * j) = acc;
}

// ------------------------------------------------------------------------------------------------
// Fused forward, quad form (the default on the encoder layout).  The forward is VALU-issue bound, and in the
// 8-lane form above every lane of a pair re-derives every sample's geometry (about 45 VALU per sample) for a
// float4 of channels.  Here a QUAD of lanes serves one (query, head) pair, lane j owning channels 4j..4j+3 and
// 16+4j..16+4j+3 (two 64-byte halves of the 128-byte row, one load address per corner: the second half is the
// immediate offset).  Lane j derives the geometry of point j of each level ONCE; the quad then takes the four
// points in turn, each lane reading the owner's corner offsets and premultiplied corner weights by DPP quad
// broadcasts (a VALU operand modifier, no LDS), so a sample costs the quad one geometry plus 4 x (4 address
// adds + 4 weight moves + 16 packed FMAs) instead of 8 x (geometry + 16 FMAs + selects).  A sample outside
// (-1, H) x (-1, W) is skipped by the exec mask (as the reference, which skips it: non-finite values at its
// clamped rows never reach the output).  Workgroup = one head of an 8 x 8 patch of queries of one level, head
// the fastest block index (each XCD's L2 gathers one head's value rows).  32-bit offsets (checked on the host).
// ------------------------------------------------------------------------------------------------
// The four points of one level for the quad forward kernels: lane j holds point j's geometry (k) and attention
// weight (wa); the quad takes the points in turn, each lane gathering its 8 channels of the point's 4 corner rows
// (addresses and weights by DPP quad broadcast) into acc0 (channels 4j..4j+3) and acc1 (16+4j..16+4j+3).
template <int PB = 2>
__device__ __forceinline__ void quad_level_fwd(const char* __restrict__ vbytes, const QuadPoint& k, float wa,
                                               unsigned cjb, f4& acc0, f4& acc1) {
  // a corner outside the level weighs 0 (its clamped row is another corner of the same sample)
  const float w1 = k.w1 * wa, w2 = k.w2 * wa, w3 = k.w3 * wa, w4 = k.w4 * wa;
  const int okb = k.ok ? 1 : 0;
  // PB points per batch: their 8 * PB loads are issued (clamped, in-level addresses) before any of their math
  constexpr int kCtrl[4] = {0x00, 0x55, 0xAA, 0xFF};
  auto batch = [&](auto first) {
    constexpr int F = decltype(first)::value;
    f4 va[PB][8];
    const char* vhi = vbytes + 64;  // the row's second half (channels 16..31): an immediate offset
    auto load = [&](f4* v, unsigned o1, unsigned o2, unsigned o3, unsigned o4) {
      v[0] = ldb4(vbytes, o1); v[1] = ldb4(vhi, o1);
      v[2] = ldb4(vbytes, o2); v[3] = ldb4(vhi, o2);
      v[4] = ldb4(vbytes, o3); v[5] = ldb4(vhi, o3);
      v[6] = ldb4(vbytes, o4); v[7] = ldb4(vhi, o4);
    };
    auto load_pt = [&](auto pp) {
      constexpr int C = kCtrl[F + decltype(pp)::value];
      load(va[decltype(pp)::value], qpermi<C>(k.o1) + cjb, qpermi<C>(k.o2) + cjb, qpermi<C>(k.o3) + cjb,
           qpermi<C>(k.o4) + cjb);
    };
    load_pt(std::integral_constant<int, 0>{});
    if constexpr (PB > 1) load_pt(std::integral_constant<int, 1>{});
    if constexpr (PB > 2) { load_pt(std::integral_constant<int, 2>{}); load_pt(std::integral_constant<int, 3>{}); }
    // pin the loads here: otherwise each point's loads sink into its exec-masked block below and the points'
    // latencies are paid one after the other
#pragma unroll
    for (int pp = 0; pp < PB; ++pp)
#pragma unroll
      for (int i = 0; i < 8; ++i) asm volatile("" : "+v"(va[pp][i]));
    auto fmas = [&](const f4* v, float u1, float u2, float u3, float u4) {
      acc0 += u1 * v[0]; acc1 += u1 * v[1];
      acc0 += u2 * v[2]; acc1 += u2 * v[3];
      acc0 += u3 * v[4]; acc1 += u3 * v[5];
      acc0 += u4 * v[6]; acc1 += u4 * v[7];
    };
    // a point outside (-1, H) x (-1, W) is skipped by the exec mask, as the reference skips it
    auto fma_pt = [&](auto pp) {
      constexpr int C = kCtrl[F + decltype(pp)::value];
      if (qpermi<C>(okb)) fmas(va[decltype(pp)::value], qpermf<C>(w1), qpermf<C>(w2), qpermf<C>(w3), qpermf<C>(w4));
    };
    fma_pt(std::integral_constant<int, 0>{});
    if constexpr (PB > 1) fma_pt(std::integral_constant<int, 1>{});
    if constexpr (PB > 2) { fma_pt(std::integral_constant<int, 2>{}); fma_pt(std::integral_constant<int, 3>{}); }
  };
  batch(std::integral_constant<int, 0>{});
  if constexpr (PB == 1) {
    batch(std::integral_constant<int, 1>{});
    batch(std::integral_constant<int, 2>{});
    batch(std::integral_constant<int, 3>{});
  } else if constexpr (PB == 2) {
    batch(std::integral_constant<int, 2>{});
  }
}

// Unfused forward, quad form (the reference op's interface: materialised sampling_loc / attention_weight, device
// spatial shapes; D = 32, P = 4, value bytes < 2^31): a quad per (n, q, m) pair, lane j reading point j of each
// level (the quad's four loc pairs / weights are contiguous).
__global__ void __launch_bounds__(256) msda_fwd_f32_q4(const float* __restrict__ value,
                                                       const int64_t* __restrict__ shapes,
                                                       const int64_t* __restrict__ lsi, const float* __restrict__ loc,
                                                       const float* __restrict__ attn, int64_t npairs, int S, int M,
                                                       int L, int Lq, float* __restrict__ out) {
  constexpr int D = 32, P = 4;
  __shared__ int sH[kMaxLevels], sW[kMaxLevels], sSt[kMaxLevels];
  if (threadIdx.x < L) {
    sH[threadIdx.x] = static_cast<int>(shapes[2 * threadIdx.x]);
    sW[threadIdx.x] = static_cast<int>(shapes[2 * threadIdx.x + 1]);
    sSt[threadIdx.x] = static_cast<int>(lsi[threadIdx.x]);
  }
  __syncthreads();
  const int64_t pair = static_cast<int64_t>(blockIdx.x) * 64 + (threadIdx.x >> 2);
  if (pair >= npairs) return;  // whole quads leave together
  const int j = threadIdx.x & 3;
  const int m = static_cast<int>(pair % M);
  const int n = static_cast<int>(pair / M / Lq);
  const int rsb = M * D * 4;
  const char* vbytes = reinterpret_cast<const char*>(value);
  const float* lp = loc + pair * L * P * 2;
  const float* ap = attn + pair * L * P;
  const unsigned cjb = 16u * j;
  f4 acc0 = {0.f, 0.f, 0.f, 0.f}, acc1 = acc0;
  for (int l = 0; l < L; ++l) {
    const int H = sH[l], W = sW[l];
    const int obase = ((n * S + sSt[l]) * M + m) * D * 4;
    const float2 xy = *reinterpret_cast<const float2*>(lp + 2 * (l * P + j));
    const QuadPoint k = quad_point(xy.y * H - 0.5f, xy.x * W - 0.5f, H, W, obase, rsb);
    quad_level_fwd(vbytes, k, ap[l * P + j], cjb, acc0, acc1);
  }
  float* o = out + pair * D + 4 * j;
  *reinterpret_cast<f4*>(o) = acc0;
  *reinterpret_cast<f4*>(o + 16) = acc1;
}

template <int LT, int PB = 2>
__global__ void __launch_bounds__(256) msda_fused_fwd_q4(const float* __restrict__ value, FrontEnd fe, TileGeom geo,
                                                         int S, int M, float* __restrict__ out) {
  constexpr int D = 32, P = 4, LP = LT * P;
  static_assert(P == 4, "one quad lane per point");
  const int qd = threadIdx.x >> 2, j = threadIdx.x & 3;
  int b = blockIdx.x;
  const int m = b % M;
  b /= M;
  int T = 0;
#pragma unroll
  for (int l = 0; l < LT; ++l) T += ((geo.H[l] + 7) >> 3) * ((geo.W[l] + 7) >> 3);
  const int n = b / T;
  int t = b - n * T, lv = 0;
#pragma unroll
  for (int l = 0; l < LT - 1; ++l) {
    const int nt = ((geo.H[l] + 7) >> 3) * ((geo.W[l] + 7) >> 3);
    if (lv == l && t >= nt) { t -= nt; lv = l + 1; }
  }
  const int Hq = geo.H[lv], Wq = geo.W[lv], tlx = (Wq + 7) >> 3;
  const int y = (t / tlx) * 8 + (qd >> 3), x = (t % tlx) * 8 + (qd & 7);
  if (y >= Hq || x >= Wq) return;  // whole quads leave together
  const int q = geo.start[lv] + y * Wq + x;
  const int64_t nq = static_cast<int64_t>(n) * S + q;
  const int rsb = M * D * 4;  // value row stride in bytes
  const char* vbytes = reinterpret_cast<const char*>(value);
  const float* prow = fe.proj + nq * fe.ld;
  const float* rrow = fe.ref + n * fe.ref_bs + static_cast<int64_t>(q) * LT * 2;
  // softmax over the pair's L*P logits (ms_deform_attn.py:103-104): lane j exps logit l*P + j of every level,
  // the quad max is exact, and every lane sums the exps in logit order (the sequential sum the backward
  // recomputes, msda_bwd_f32_tiled), so the attention weights are bit-identical to the other kernels'
  const float* lg = prow + fe.lg0(m, M, LP);
  float e[LT];
  float mx = -INFINITY;
#pragma unroll
  for (int l = 0; l < LT; ++l) { e[l] = lg[l * P + j]; mx = fmaxf(mx, e[l]); }
  mx = fmaxf(mx, qpermf<0xB1>(mx));
  mx = fmaxf(mx, qpermf<0x4E>(mx));
  float sum = 0.f;
#pragma unroll
  for (int l = 0; l < LT; ++l) {
    e[l] = expf(e[l] - mx);
    sum += qpermf<0x00>(e[l]);
    sum += qpermf<0x55>(e[l]);
    sum += qpermf<0xAA>(e[l]);
    sum += qpermf<0xFF>(e[l]);
  }
  const float inv = 1.f / sum;
  const f4 z = {0.f, 0.f, 0.f, 0.f};
  f4 acc0 = z, acc1 = z;
  const unsigned cjb = 16u * j;  // this lane's channel bytes within a row half
  auto level = [&](int l, auto pow2) {
    constexpr bool POW2 = decltype(pow2)::value;
    const int H = geo.H[l], W = geo.W[l];
    const int obase = ((n * S + geo.start[l]) * M + m) * D * 4;
    const float2 rf = *reinterpret_cast<const float2*>(rrow + 2 * l);
    const float2 off = *reinterpret_cast<const float2*>(prow + fe.off0(m, LP) + (l * P + j) * 2);
    const float sx = rf.x + div_norm(off.x, static_cast<float>(W), geo.invW[l], POW2);
    const float sy = rf.y + div_norm(off.y, static_cast<float>(H), geo.invH[l], POW2);
    // this lane's point: corner byte offsets and weights (a corner outside the level weighted 0: its clamped row
    // is another corner of the same sample), times the attention weight
    const QuadPoint k = quad_point(sy * H - 0.5f, sx * W - 0.5f, H, W, obase, rsb);
    quad_level_fwd<PB>(vbytes, k, e[l] * inv, cjb, acc0, acc1);
  };
#pragma unroll
  for (int l = 0; l < LT; ++l) {
    if (((geo.W[l] & (geo.W[l] - 1)) | (geo.H[l] & (geo.H[l] - 1))) == 0) level(l, std::true_type{});
    else level(l, std::false_type{});
  }
  float* o = out + (nq * M + m) * D + 4 * j;
  *reinterpret_cast<f4*>(o) = acc0;
  *reinterpret_cast<f4*>(o + 16) = acc1;
}

// ------------------------------------------------------------------------------------------------
// Fused forward with LDS-staged value windows (the default on the encoder layout).
//
// The quad kernel above gathers every sample's four 128-byte corner rows through the texture path (L1,
// 64 B/clk/CU): 16.9 GB per config-2 launch, which bounds it.  Neighbouring queries sample one neighbourhood,
// so here a workgroup takes one head of one spatial tile -- the same normalised rectangle on every level (8 x 16
// pixels on the finest), its queries drawn from all levels -- and, level by level:
//   1. each quad lane derives its point's geometry for its queries (three rounds of 64 queries), and the
//      workgroup reduces the touched corners to a box;
//   2. the box, clipped to the tile +- msda_fwd_halo and shrunk until it fits msda_fwd_cap rows, is copied into
//      LDS by LDS-DMA (global_load_lds_dwordx4, 8 whole rows per wave-instruction, no VGPRs), once;
//   3. the quads read their corners with ds_read_b128 (256 B/clk/CU), a sample whose corners leave the window
//      reading them from HBM as before.
// Rows sit at a 128-byte stride with the two 64-byte halves of row r swapped when bit 1 of r is set, so the four
// quads of a ds_read_b128 lane group (a wave's quads are consecutive queries) read four distinct bank quarters
// when their samples lie in consecutive window rows; the swizzle is applied on the DMA's per-lane source address.
// Arithmetic per sample and per output element is the quad kernel's, in the same order (same results bit for bit).
// ------------------------------------------------------------------------------------------------
constexpr int kFwdLdsThreads = 256;
constexpr int kFwdLdsRounds = 3;   // queries per workgroup <= 3 * 64
constexpr int kFwdLdsCap = 416;    // window rows at most: 52 KB + the boxes, three workgroups per CU (145 VGPRs: three
                                   // waves per SIMD; a four-wave build spills 16 registers and measured 0.635 vs 0.60 ms)
constexpr int kFwdWinRows = kFwdLdsCap - 8;  // window rows the host may ask for: the last 1 KB block is the zero row

// b_i = (quad lane C's a_i) + c for the four corners, as v_add_u32_dpp (hipcc leaves the DPP broadcast and the add
// apart when the broadcast source comes out of a select).  The s_nop covers the DPP read-after-VALU-write hazard,
// which the compiler's hazard recognizer does not see inside inline asm.
template <int C>
__device__ __forceinline__ void dpp_add4(unsigned& b1, unsigned& b2, unsigned& b3, unsigned& b4, unsigned a1, unsigned a2,
                                         unsigned a3, unsigned a4, unsigned c) {
#define M2F_DPP4(QP)                                                                                         \
  asm("s_nop 1\n\t"                                                                                          \
      "v_add_u32_dpp %0, %4, %8 quad_perm:" QP " row_mask:0xf bank_mask:0xf bound_ctrl:1\n\t"                \
      "v_add_u32_dpp %1, %5, %8 quad_perm:" QP " row_mask:0xf bank_mask:0xf bound_ctrl:1\n\t"                \
      "v_add_u32_dpp %2, %6, %8 quad_perm:" QP " row_mask:0xf bank_mask:0xf bound_ctrl:1\n\t"                \
      "v_add_u32_dpp %3, %7, %8 quad_perm:" QP " row_mask:0xf bank_mask:0xf bound_ctrl:1"                     \
      : "=&v"(b1), "=&v"(b2), "=&v"(b3), "=&v"(b4)                                                            \
      : "v"(a1), "v"(a2), "v"(a3), "v"(a4), "v"(c))
  if constexpr (C == 0x00) M2F_DPP4("[0,0,0,0]");
  else if constexpr (C == 0x55) M2F_DPP4("[1,1,1,1]");
  else if constexpr (C == 0xAA) M2F_DPP4("[2,2,2,2]");
  else M2F_DPP4("[3,3,3,3]");
#undef M2F_DPP4
}

// The four points of one level for one query: lane j of the quad owns point j (mode md: 0 = skipped (nothing read),
// 1 = corners in the LDS window at byte offsets a1..a4 (first-half bases, win_row), 2 = corners in HBM at byte
// offsets a1..a4);
// weights premultiplied by the attention weight, a corner outside the level weighted 0.
__device__ __forceinline__ void quad_gather_win(const char* __restrict__ vbytes,
                                                const __attribute__((address_space(3))) unsigned char* win, int md,
                                                unsigned a1, unsigned a2, unsigned a3, unsigned a4, float w1, float w2,
                                                float w3, float w4, unsigned cjb, f4& acc0, f4& acc1) {
  constexpr int kCtrl[4] = {0x00, 0x55, 0xAA, 0xFF};
  auto batch = [&](auto first) {
    constexpr int F = decltype(first)::value;
    f4 va[2][8];
    int mdp[2];
    auto load_pt = [&](auto pp) {
      constexpr int I = decltype(pp)::value, C = kCtrl[F + I];
      const int mq = qpermi<C>(md);
      unsigned b1, b2, b3, b4;
      dpp_add4<C>(b1, b2, b3, b4, a1, a2, a3, a4, cjb);
      mdp[I] = mq;
      f4* v = va[I];
      if (mq == 2) {
        const char* vhi = vbytes + 64;
        v[0] = ldb4(vbytes, b1); v[1] = ldb4(vhi, b1);
        v[2] = ldb4(vbytes, b2); v[3] = ldb4(vhi, b2);
        v[4] = ldb4(vbytes, b3); v[5] = ldb4(vhi, b3);
        v[6] = ldb4(vbytes, b4); v[7] = ldb4(vhi, b4);
      } else if (mq == 1) {  // the second half of a window row is 512 bytes on (an offset field of the read)
        // an address-space-3 load: with generic pointers the compiler merges the two branches' loads into one flat
        // load of a selected 64-bit address
        auto lds4 = [&](unsigned o) { return *(const __attribute__((address_space(3))) f4*)(win + o); };
        v[0] = lds4(b1); v[1] = lds4(b1 + 512u);
        v[2] = lds4(b2); v[3] = lds4(b2 + 512u);
        v[4] = lds4(b3); v[5] = lds4(b3 + 512u);
        v[6] = lds4(b4); v[7] = lds4(b4 + 512u);
      }
    };
    load_pt(std::integral_constant<int, 0>{});
    load_pt(std::integral_constant<int, 1>{});
#pragma unroll
    for (int pp = 0; pp < 2; ++pp)
#pragma unroll
      for (int i = 0; i < 8; ++i) asm volatile("" : "+v"(va[pp][i]));
    auto fma_pt = [&](auto pp) {
      constexpr int I = decltype(pp)::value, C = kCtrl[F + I];
      const float u1 = qpermf<C>(w1), u2 = qpermf<C>(w2), u3 = qpermf<C>(w3), u4 = qpermf<C>(w4);
      if (mdp[I] != 0) {
        const f4* v = va[I];
        acc0 += u1 * v[0]; acc1 += u1 * v[1];
        acc0 += u2 * v[2]; acc1 += u2 * v[3];
        acc0 += u3 * v[4]; acc1 += u3 * v[5];
        acc0 += u4 * v[6]; acc1 += u4 * v[7];
      }
    };
    fma_pt(std::integral_constant<int, 0>{});
    fma_pt(std::integral_constant<int, 1>{});
  };
  batch(std::integral_constant<int, 0>{});
  batch(std::integral_constant<int, 2>{});
}

// quad_gather_win when no lane of the wave reads HBM this round and level (the common case): every lane's corners
// are window rows, a skipped point's the kernel's zero row (zero weights times zeros add +0), so there is no mode
// broadcast, compare or branch per point
__device__ __forceinline__ void quad_gather_lds(const __attribute__((address_space(3))) unsigned char* win, unsigned a1,
                                                unsigned a2, unsigned a3, unsigned a4, float w1, float w2, float w3,
                                                float w4, unsigned cjb, f4& acc0, f4& acc1) {
  constexpr int kCtrl[4] = {0x00, 0x55, 0xAA, 0xFF};
  auto lds4 = [&](unsigned o) { return *(const __attribute__((address_space(3))) f4*)(win + o); };
  auto batch = [&](auto first) {
    constexpr int F = decltype(first)::value;
    f4 va[2][8];
    auto load_pt = [&](auto pp) {
      constexpr int I = decltype(pp)::value, C = kCtrl[F + I];
      unsigned b1, b2, b3, b4;
      dpp_add4<C>(b1, b2, b3, b4, a1, a2, a3, a4, cjb);
      f4* v = va[I];
      v[0] = lds4(b1); v[1] = lds4(b1 + 512u);
      v[2] = lds4(b2); v[3] = lds4(b2 + 512u);
      v[4] = lds4(b3); v[5] = lds4(b3 + 512u);
      v[6] = lds4(b4); v[7] = lds4(b4 + 512u);
    };
    load_pt(std::integral_constant<int, 0>{});
    load_pt(std::integral_constant<int, 1>{});
    auto fma_pt = [&](auto pp) {
      constexpr int I = decltype(pp)::value, C = kCtrl[F + I];
      const float u1 = qpermf<C>(w1), u2 = qpermf<C>(w2), u3 = qpermf<C>(w3), u4 = qpermf<C>(w4);
      const f4* v = va[I];
      acc0 += u1 * v[0]; acc1 += u1 * v[1];
      acc0 += u2 * v[2]; acc1 += u2 * v[3];
      acc0 += u3 * v[4]; acc1 += u3 * v[5];
      acc0 += u4 * v[6]; acc1 += u4 * v[7];
    };
    fma_pt(std::integral_constant<int, 0>{});
    fma_pt(std::integral_constant<int, 1>{});
  };
  batch(std::integral_constant<int, 0>{});
  batch(std::integral_constant<int, 2>{});
}

// wave-wide min / max by DPP (no LDS round trips, unlike __shfl_xor's ds_bpermute): the four intra-row steps leave
// every lane with its 16-lane row's result, row_bcast:15 / :31 fold the rows into lane 63, read out uniformly
template <bool MAX>
__device__ __forceinline__ int wave_minmax(int v) {
  constexpr int id = MAX ? INT_MIN : INT_MAX;
  auto op = [](int a, int b) { return MAX ? max(a, b) : min(a, b); };
  v = op(v, __builtin_amdgcn_update_dpp(id, v, 0xB1, 0xF, 0xF, false));    // quad_perm [1,0,3,2]
  v = op(v, __builtin_amdgcn_update_dpp(id, v, 0x4E, 0xF, 0xF, false));    // quad_perm [2,3,0,1]
  v = op(v, __builtin_amdgcn_update_dpp(id, v, 0x141, 0xF, 0xF, false));   // row_half_mirror
  v = op(v, __builtin_amdgcn_update_dpp(id, v, 0x140, 0xF, 0xF, false));   // row_mirror
  v = op(v, __builtin_amdgcn_update_dpp(id, v, 0x142, 0xA, 0xF, false));   // row_bcast:15 into rows 1, 3
  v = op(v, __builtin_amdgcn_update_dpp(id, v, 0x143, 0xC, 0xF, false));   // row_bcast:31 into rows 2, 3
  return __builtin_amdgcn_readlane(v, 63);
}

// Window rows in 1 KB blocks of 8 (one LDS-DMA instruction each): row r's first 64-byte half at block (r >> 3), slot
// r & 7 of the block's first 512 bytes, its second half 512 bytes on.  A quad's 64-byte read of either half lands in
// bank quarter r & 3, as with the previous in-row half swap (x-adjacent queries at one scale: distinct quarters), and
// the second half is a constant offset instead of an address xor per corner.  win_row: the first half's byte base.
__device__ __forceinline__ unsigned win_row(int r) {
  return (static_cast<unsigned>(r >> 3) << 10) | (static_cast<unsigned>(r & 7) << 6);
}

// block -> (image * tiles + tile, head).  Blocks are dealt to the 8 XCDs round-robin.  Default: the head fastest,
// so XCD x gathers head x's value rows.  xcdmap (msda_fwd_xcd=1): XCD x takes the x-th eighth of the (image, tile)
// list, every head of a tile in turn, so a query's projection row (its heads' offsets and logits share 128-byte
// lines) is fetched into one L2 (config 2: FETCH -15 %, WRITE +29 %, time unchanged: not the default).
__device__ __forceinline__ void fwd_block(const TileGeom& geo, int M, int& m, int& b) {
  if (geo.xcdmap) {
    const int s = static_cast<int>(blockIdx.x >> 3), x = static_cast<int>(blockIdx.x & 7u);
    m = s % M;
    b = x * static_cast<int>(gridDim.x / (8u * static_cast<unsigned>(M))) + s / M;
  } else {
    m = static_cast<int>(blockIdx.x % static_cast<unsigned>(M));
    b = static_cast<int>(blockIdx.x / static_cast<unsigned>(M));
  }
}

// FUSED: the samples come from the projection and the reference points (fe); otherwise (the reference op's
// interface, m2f_msda_fwd_f32) from materialised sampling locations loc (N, S, M, L, P, 2) and attention weights
// attn (N, S, M, L, P), the encoder layout (query i at pyramid position i; host shapes).
template <int LT, bool FUSED = true>
__global__ void __launch_bounds__(kFwdLdsThreads, 3) msda_fused_fwd_lds(const float* __restrict__ value, FrontEnd fe,
                                                                      TileGeom geo, int S, int M,
                                                                      float* __restrict__ out,
                                                                      const float* __restrict__ loc = nullptr,
                                                                      const float* __restrict__ attn = nullptr) {
  constexpr int D = 32, P = 4, LP = LT * P, R = kFwdLdsRounds, NW = kFwdLdsThreads / 64;
  // one static array (a constant base folds into the ds_read addresses): window rows | per-wave boxes [LT][NW]
  __shared__ __attribute__((aligned(16))) unsigned char smem[kFwdLdsCap * 128 + kTileMaxL * NW * 16];
  const int cap = geo.max_rows;  // window rows in use (a multiple of 8, <= kFwdLdsCap)
  int4* bbw = reinterpret_cast<int4*>(smem + kFwdLdsCap * 128);
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6, j = lane & 3;
  // the zero row (window row kFwdWinRows, beyond every window): the LDS-only gather's skipped points read it
  if (tid < 64) reinterpret_cast<f4*>(smem + kFwdWinRows * 128)[tid] = f4{0.f, 0.f, 0.f, 0.f};   // before any barrier
  const int ntiles = geo.nty * geo.ntx;
  int m, b;
  fwd_block(geo, M, m, b);
  const int n = b / ntiles, tile = b - n * ntiles;
  const int ty = tile / geo.ntx, tx = tile - ty * geo.ntx;
  int qy0[LT], qy1[LT], qx0[LT], qx1[LT], qc[LT + 1];
  qc[0] = 0;
#pragma unroll
  for (int l = 0; l < LT; ++l) {
    qy0[l] = tile_lo(ty, geo.H[l], geo.nty); qy1[l] = tile_lo(ty + 1, geo.H[l], geo.nty);
    qx0[l] = tile_lo(tx, geo.W[l], geo.ntx); qx1[l] = tile_lo(tx + 1, geo.W[l], geo.ntx);
    qc[l + 1] = qc[l] + (qy1[l] - qy0[l]) * (qx1[l] - qx0[l]);
  }
  const int Qt = qc[LT];
  const char* vbytes = reinterpret_cast<const char*>(value);
  const int rsb = M * D * 4;  // value row stride in bytes; value bytes < 2^31 (host check)
  unsigned cjb = 16u * j;
  asm volatile("" : "+v"(cjb));  // materialised once, here: the corner broadcasts then fold into v_add_u32_dpp
  // byte offsets from the kernarg bases are 32-bit (proj, ref, value and out under 2^31 bytes: host check)
  const char* pbytes = reinterpret_cast<const char*>(fe.proj);
  const char* rbytes = reinterpret_cast<const char*>(fe.ref) + static_cast<int64_t>(n) * fe.ref_bs * 4;
  const unsigned pld = static_cast<unsigned>(fe.ld) * 4u;
  // this quad's query in each round: the tile's queries level by level, row-major in each level's rectangle
  int qpos[R];
  unsigned vmask = 0u;  // bit r: round r's query exists
  float wa[R][LT];
#pragma unroll
  for (int r = 0; r < R; ++r) {
    const int qi = r * (kFwdLdsThreads / 4) + (tid >> 2);
    vmask |= qi < Qt ? 1u << r : 0u;
    const int qq = min(qi, Qt - 1);
    int lq = 0;
#pragma unroll
    for (int l = 1; l < LT; ++l) lq = qq >= qc[l] ? l : lq;
    int qb = 0, qw = 1, y0 = 0, x0 = 0, W = 1;
#pragma unroll
    for (int l = 0; l < LT; ++l)
      if (l == lq) { qb = qc[l]; qw = qx1[l] - qx0[l]; y0 = qy0[l]; x0 = qx0[l]; W = geo.W[l]; }
    const int rr = qq - qb;
    // rr / qw by the reciprocal ((rr + 0.5) / qw is >= 0.5 / qw from an integer; rr < 2^16)
    const int yy = static_cast<int>((static_cast<float>(rr) + 0.5f) * __builtin_amdgcn_rcpf(static_cast<float>(qw)));
    const int xx = rr - yy * qw;
    int st = 0;
#pragma unroll
    for (int l = 0; l < LT; ++l) st = l == lq ? geo.start[l] : st;
    qpos[r] = st + (y0 + yy) * W + x0 + xx;
  }
  // every round's logits are loaded before any round's softmax: written inside the round loop, each round's loads
  // were waited on before the next round's were issued (ISA), three memory round trips instead of one
  float el[R][LT];
  if constexpr (FUSED) {
    // the byte offsets first, materialised (else the first load's destination is reused in the next round's 64-bit
    // address arithmetic and waited on)
    unsigned lgb[R];
#pragma unroll
    for (int r = 0; r < R; ++r) {
      lgb[r] = static_cast<unsigned>(n * S + qpos[r]) * pld + static_cast<unsigned>(fe.lg0(m, M, LP) + j) * 4u;
      asm volatile("" : "+v"(lgb[r]));
    }
#pragma unroll
    for (int r = 0; r < R; ++r)
#pragma unroll
      for (int l = 0; l < LT; ++l) el[r][l] = *reinterpret_cast<const float*>(pbytes + lgb[r] + l * P * 4);
  }
#pragma unroll
  for (int r = 0; r < R; ++r) {
    if constexpr (!FUSED) break;  // the attention weights are read per level
    // softmax over the pair's L*P logits, exactly as msda_fused_fwd_q4 (and the backward's recomputation)
    float e[LT];
    float mx = -INFINITY;
#pragma unroll
    for (int l = 0; l < LT; ++l) {
      e[l] = el[r][l];
      mx = fmaxf(mx, e[l]);
    }
    mx = fmaxf(mx, qpermf<0xB1>(mx));
    mx = fmaxf(mx, qpermf<0x4E>(mx));
    float sum = 0.f;
#pragma unroll
    for (int l = 0; l < LT; ++l) {
      e[l] = expf(e[l] - mx);
      sum += qpermf<0x00>(e[l]);
      sum += qpermf<0x55>(e[l]);
      sum += qpermf<0xAA>(e[l]);
      sum += qpermf<0xFF>(e[l]);
    }
    const float inv = 1.f / sum;
#pragma unroll
    for (int l = 0; l < LT; ++l) wa[r][l] = e[l] * inv;
  }
  const f4 z = {0.f, 0.f, 0.f, 0.f};
  f4 acc0[R], acc1[R];
#pragma unroll
  for (int r = 0; r < R; ++r) { acc0[r] = z; acc1[r] = z; }

#pragma unroll
  for (int l = 0; l < LT; ++l) {
    const int H = geo.H[l], W = geo.W[l];
    const int lbase = ((n * S + geo.start[l]) * M + m) * D * 4;
    // the level's loads hang on an opaque zero defined here, after the previous level's gather: otherwise the
    // compiler hoists every level's loads to the kernel's start and spills
    int zq = 0;
    asm volatile("" : "+v"(zq));
    // 1. lane j's point (l, j) of each round's query: corner block (y0, x0) clamped into the level, whether the
    //    +1 row / column is a corner inside the level (ey, ex), the four weights (x attention weight), ok
    int gy[R], gx[R], gfl[R];
    float gw[R][4];
    int bmin_y = 0x7fffffff, bmax_y = -1, bmin_x = 0x7fffffff, bmax_x = -1;
    auto geometry = [&](auto pow2) {
      constexpr bool POW2 = decltype(pow2)::value;
      const float fH = static_cast<float>(H), fW = static_cast<float>(W);
      const float fHm1 = static_cast<float>(H - 1), fWm1 = static_cast<float>(W - 1);
      // every round's loads first: the per-round asm pins below are scheduling barriers, so loads written inside the
      // round loop were waited on round by round
      float2 rfs[R], offs[R];
#pragma unroll
      for (int r = 0; r < R; ++r) {
        if constexpr (FUSED) {
          const unsigned rfb = static_cast<unsigned>((qpos[r] + zq) * LT + l) * 8u;
          const unsigned ofb = static_cast<unsigned>(n * S + qpos[r] + zq) * pld + static_cast<unsigned>(fe.off0(m, LP) + (l * P + j) * 2) * 4u;
          rfs[r] = *reinterpret_cast<const float2*>(rbytes + rfb);
          offs[r] = *reinterpret_cast<const float2*>(pbytes + ofb);
        } else {
          const unsigned ki = static_cast<unsigned>(((n * S + qpos[r] + zq) * M + m) * LP + l * P + j);
          offs[r] = *reinterpret_cast<const float2*>(reinterpret_cast<const char*>(loc) + ki * 8u);
          wa[r][l] = *reinterpret_cast<const float*>(reinterpret_cast<const char*>(attn) + ki * 4u);
        }
      }
#pragma unroll
      for (int r = 0; r < R; ++r) {
        float sx, sy;
        if constexpr (FUSED) {
          sx = rfs[r].x + div_norm(offs[r].x, fW, geo.invW[l], POW2);
          sy = rfs[r].y + div_norm(offs[r].y, fH, geo.invH[l], POW2);
        } else {
          sx = offs[r].x;
          sy = offs[r].y;
        }
        const float h = sy * H - 0.5f, w = sx * W - 0.5f;
        const bool ok = ((vmask >> r) & 1u) && h > -1.f && w > -1.f && h < fH && w < fW;
        const float hs = ok ? h : -2.f, ws = ok ? w : -2.f;
        const float fh = floorf(hs), fw = floorf(ws);
        const float ly = hs - fh, lx = ws - fw, hy = 1.f - ly, hx = 1.f - lx;
        const bool vy0 = fh >= 0.f, vy1 = fh < fHm1, vx0 = fw >= 0.f, vx1 = fw < fWm1;
        const int y0 = static_cast<int>(__builtin_amdgcn_fmed3f(fh, 0.f, fHm1));
        const int x0 = static_cast<int>(__builtin_amdgcn_fmed3f(fw, 0.f, fWm1));
        const int ey = (vy0 && vy1) ? 1 : 0, ex = (vx0 && vx1) ? 1 : 0;
        const float a = wa[r][l];
        gw[r][0] = (vy0 && vx0) ? hy * hx * a : 0.f;
        gw[r][1] = (vy0 && vx1) ? hy * lx * a : 0.f;
        gw[r][2] = (vy1 && vx0) ? ly * hx * a : 0.f;
        // a skipped point (hs = ws = -2) has vy0 = vx0 = false, so only corner 4 needs ok: its LDS-only gather still
        // runs the FMAs (on the zero row), and 0 * 0 * a would carry a NaN weight into the output
        gw[r][3] = (ok && vy1 && vx1) ? ly * lx * a : 0.f;
        gy[r] = y0;
        gx[r] = x0;
        gfl[r] = (ok ? 1 : 0) | (ey << 1) | (ex << 2);
        // materialised here: left to the compiler, the weights sink past the barriers into the gather and their
        // inputs (fractions, corner masks) stay live instead
        asm volatile("" : "+v"(gw[r][0]), "+v"(gw[r][1]), "+v"(gw[r][2]), "+v"(gw[r][3]), "+v"(gy[r]), "+v"(gx[r]),
                     "+v"(gfl[r]));
        if (ok) {
          bmin_y = min(bmin_y, y0); bmax_y = max(bmax_y, y0 + ey);
          bmin_x = min(bmin_x, x0); bmax_x = max(bmax_x, x0 + ex);
        }
      }
    };
    if (FUSED && ((W & (W - 1)) | (H & (H - 1))) == 0) geometry(std::true_type{});
    else geometry(std::false_type{});
    bmin_y = wave_minmax<false>(bmin_y); bmax_y = wave_minmax<true>(bmax_y);
    bmin_x = wave_minmax<false>(bmin_x); bmax_x = wave_minmax<true>(bmax_x);
    if (lane == 0) bbw[l * NW + wid] = make_int4(bmin_y, bmax_y, bmin_x, bmax_x);
    __syncthreads();  // the boxes are in; every wave is done reading the previous level's window
    // 2. the window: the box clipped to the tile +- halo, the halo shrinking until the rows fit (uniform)
    int by0 = 0x7fffffff, by1 = -1, bx0 = 0x7fffffff, bx1 = -1;
#pragma unroll
    for (int w = 0; w < NW; ++w) {
      const int4 t = bbw[l * NW + w];
      by0 = min(by0, t.x); by1 = max(by1, t.y); bx0 = min(bx0, t.z); bx1 = max(bx1, t.w);
    }
    by0 = __builtin_amdgcn_readfirstlane(by0); by1 = __builtin_amdgcn_readfirstlane(by1);
    bx0 = __builtin_amdgcn_readfirstlane(bx0); bx1 = __builtin_amdgcn_readfirstlane(bx1);
    int wy0 = 0, wy1 = -1, wx0 = 0, wx1 = -1;
    for (int halo = geo.max_halo; halo >= 0 && by1 >= 0; --halo) {
      wy0 = max(by0, qy0[l] - halo); wy1 = min(by1, qy1[l] - 1 + halo);
      wx0 = max(bx0, qx0[l] - halo); wx1 = min(bx1, qx1[l] - 1 + halo);
      if (wy1 < wy0 || wx1 < wx0) { wy1 = wy0 - 1; break; }
      if ((wy1 - wy0 + 1) * (wx1 - wx0 + 1) <= cap) break;
      if (halo == 0) wy1 = wy0 - 1;  // the tile itself does not fit (the host sizes cap so it does): no window
    }
    const int wh = wy1 >= wy0 ? wy1 - wy0 + 1 : 0, ww = wh > 0 ? wx1 - wx0 + 1 : 0;
    const int rows = wh * ww;
    {
      const float iww = ww > 0 ? 1.f / static_cast<float>(ww) : 0.f;
      const int nblk = (rows + 7) >> 3;
      for (int blk = wid; blk < nblk; blk += NW) {
        // lane l fills block slot l: row blk * 8 + ((l >> 2) & 7), 16-byte chunk (l >> 5) * 4 + (l & 3) of it
        const int r = min(blk * 8 + ((lane >> 2) & 7), rows - 1);
        const int yy = static_cast<int>((static_cast<float>(r) + 0.5f) * iww), xx = r - yy * ww;
        const unsigned c = static_cast<unsigned>(((lane >> 5) << 2) | (lane & 3));
        const unsigned goff = static_cast<unsigned>(mad_u24((wy0 + yy) * W + wx0 + xx, rsb, lbase)) + 16u * c;
        __builtin_amdgcn_global_load_lds(reinterpret_cast<const void*>(vbytes + goff),
                                         (__attribute__((address_space(3))) void*)(smem + blk * 1024),
                                         16, 0, 0);
      }
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }
    __syncthreads();  // the window is in LDS
    // 3. gather: window corners from LDS, the rest from HBM
#pragma unroll
    for (int r = 0; r < R; ++r) {
      const int fl = gfl[r], y0 = gy[r], x0 = gx[r];
      const int ey = (fl >> 1) & 1, ex = (fl >> 2) & 1;
      const bool ok = fl & 1;
      const bool inwin = ok && y0 >= wy0 && y0 + ey <= wy1 && x0 >= wx0 && x0 + ex <= wx1;
      const int md = ok ? (inwin ? 1 : 2) : 0;
      const auto* win = (const __attribute__((address_space(3))) unsigned char*)smem;
      // wave-uniform: window rows only (the op-level build, FUSED = false, keeps the general path: with both it spills)
      if (FUSED && !__any(md == 2)) {
        // a skipped point's corners all on the zero row (row index kFwdWinRows, no +1 row / column)
        const int q1 = inwin ? (y0 - wy0) * ww + (x0 - wx0) : kFwdWinRows;
        const int qx = inwin ? ex : 0, q3 = q1 + (inwin && ey ? ww : 0);
        quad_gather_lds(win, win_row(q1), win_row(q1 + qx), win_row(q3), win_row(q3 + qx), gw[r][0], gw[r][1],
                        gw[r][2], gw[r][3], cjb, acc0[r], acc1[r]);
      } else {
        // both address forms, then a select (straight-line code keeps the broadcasts foldable into v_add_u32_dpp)
        const int r1 = (y0 - wy0) * ww + (x0 - wx0), r3 = r1 + (ey ? ww : 0);
        const unsigned g1 = static_cast<unsigned>(mad_u24(mad_u24(y0, W, x0), rsb, lbase));
        const unsigned dx = ex ? rsb : 0u, dy = ey ? static_cast<unsigned>(W * rsb) : 0u;
        const unsigned a1 = inwin ? win_row(r1) : g1, a2 = inwin ? win_row(r1 + ex) : g1 + dx;
        const unsigned a3 = inwin ? win_row(r3) : g1 + dy, a4 = inwin ? win_row(r3 + ex) : g1 + dy + dx;
        quad_gather_win(vbytes, win, md, a1, a2, a3, a4, gw[r][0], gw[r][1], gw[r][2], gw[r][3], cjb, acc0[r], acc1[r]);
      }
      if constexpr (!FUSED) asm volatile("" ::: "memory");  // one round's gather at a time (else the scheduler
                                                             // overlaps rounds and spills)
    }
  }
#pragma unroll
  for (int r = 0; r < R; ++r) {
    if (!((vmask >> r) & 1u)) continue;
    char* o = reinterpret_cast<char*>(out) + (static_cast<unsigned>((n * S + qpos[r]) * M + m) * 128u + cjb);
    *reinterpret_cast<f4*>(o) = acc0[r];
    *reinterpret_cast<f4*>(o + 64) = acc1[r];
  }
}

// ------------------------------------------------------------------------------------------------
// Fused forward, two lanes per (query, head) (msda_fwd_pair=1; measured and not the default: 0.535-0.542 ms against
// the quad-per-query LDS-window kernel's 0.519-0.531 at config 2 near-init, 0.85 against 0.77 ms under N(0, 4 px),
// profiles/r06_o_msda_fwd_pair_ab.txt).
//
// The LDS-window kernel above runs a lane quad per query: lane j derives point j's geometry and every lane gathers
// 8 channels of each point, so a point costs each lane 8 DPP broadcasts (4 corner addresses, 4 weights) for 16
// packed FMAs, and a workgroup holds 3 rounds of 64 queries whose geometry and accumulators stay live across the
// gathers (146 VGPRs: three workgroups per CU).  Here lane h of a pair owns channels 8k + 4h .. 8k + 4h + 3 (k < 4)
// of its query and points 2h and 2h+1 of each level: a point costs 8 broadcasts for 32 packed FMAs (a corner's 64 bytes are four
// ds_read_b128 off one address), a workgroup takes one round of 128 queries (8 x 12 finest-level tiles) and needs
// 138 VGPRs (three workgroups per CU; four at 128 VGPRs with a few spills).  Banking: a ds_read_b128 serves 16 lanes per LDS cycle (MI355X_MICROARCH.md
// §LDS), here 8 pairs, so the 8 pairs of each lane group take 8 consecutive queries (x-adjacent, so their corner
// rows are too), and the window holds rows in 1 KB blocks of 8 whose 32-byte pieces k sit in line k (256 bytes)
// at (row & 7) * 32: at each step the group's 8 pairs read 8 distinct 32-byte bank slots when their rows are 8
// consecutive window rows (lane h: the piece's 16 bytes at +16h, channels 8k + 4h .. 8k + 4h + 3).  Window
// staging, the HBM path for corners outside the window and the zero row for skipped points are the LDS-window
// kernel's; every output element is accumulated in the quad kernel's order (levels, points, corners), so the
// output is the quad kernel's bit for bit.
// ------------------------------------------------------------------------------------------------
constexpr int kFwdPairThreads = 256;
constexpr int kFwdPairQueries = kFwdPairThreads / 2;
#ifndef M2F_FWD_PAIR_WGS
#define M2F_FWD_PAIR_WGS 3  // workgroups per CU, 416-row windows (4 with 312-row windows: 128 VGPRs, 11 spilled,
                            // 0.537-0.553 vs 0.535-0.542 ms)
#endif
constexpr int kFwdPairWgs = M2F_FWD_PAIR_WGS;
constexpr int kFwdPairCap = kFwdPairWgs == 4 ? 312 : 416;  // window rows incl. the zero row's 1 KB block
constexpr int kFwdPairWinRows = kFwdPairCap - 8;
static_assert(kFwdPairWgs * (kFwdPairCap * 128 + kTileMaxL * 4 * 16) <= 160 * 1024, "pair forward LDS per CU");

// pair broadcasts: quad_perm [0,0,2,2] (lane 0 of each pair) or [1,1,3,3] (lane 1)
template <int HS>
__device__ __forceinline__ float pbcast(float v) { return qpermf<HS ? 0xF5 : 0xA0>(v); }
template <int HS>
__device__ __forceinline__ int pbcasti(int v) { return qpermi<HS ? 0xF5 : 0xA0>(v); }

// b_i = (pair lane HS's a_i) + c, as v_add_u32_dpp (see dpp_add4)
template <int HS>
__device__ __forceinline__ void dpp_add4p(unsigned& b1, unsigned& b2, unsigned& b3, unsigned& b4, unsigned a1,
                                          unsigned a2, unsigned a3, unsigned a4, unsigned c) {
#define M2F_DPP4P(QP)                                                                                        \
  asm("s_nop 1\n\t"                                                                                          \
      "v_add_u32_dpp %0, %4, %8 quad_perm:" QP " row_mask:0xf bank_mask:0xf bound_ctrl:1\n\t"                \
      "v_add_u32_dpp %1, %5, %8 quad_perm:" QP " row_mask:0xf bank_mask:0xf bound_ctrl:1\n\t"                \
      "v_add_u32_dpp %2, %6, %8 quad_perm:" QP " row_mask:0xf bank_mask:0xf bound_ctrl:1\n\t"                \
      "v_add_u32_dpp %3, %7, %8 quad_perm:" QP " row_mask:0xf bank_mask:0xf bound_ctrl:1"                     \
      : "=&v"(b1), "=&v"(b2), "=&v"(b3), "=&v"(b4)                                                            \
      : "v"(a1), "v"(a2), "v"(a3), "v"(a4), "v"(c))
  if constexpr (HS == 0) M2F_DPP4P("[0,0,2,2]");
  else M2F_DPP4P("[1,1,3,3]");
#undef M2F_DPP4P
}

// window layout of the pair kernel: row r's piece k (bytes 32k .. 32k + 31) at pwin_row(r) + 256k
__device__ __forceinline__ unsigned pwin_row(int r) {
  return (static_cast<unsigned>(r >> 3) << 10) | (static_cast<unsigned>(r & 7) << 5);
}

template <int LT>
__global__ void __launch_bounds__(kFwdPairThreads, kFwdPairWgs) msda_fused_fwd_pair(const float* __restrict__ value,
                                                                                   FrontEnd fe, TileGeom geo, int S,
                                                                                   int M, float* __restrict__ out) {
  constexpr int D = 32, P = 4, LP = LT * P, NW = kFwdPairThreads / 64;
  // window rows | per-wave boxes [LT][NW]
  __shared__ __attribute__((aligned(16))) unsigned char smem[kFwdPairCap * 128 + kTileMaxL * NW * 16];
  const int cap = geo.max_rows;  // window rows in use (a multiple of 8, <= kFwdPairWinRows)
  int4* bbw = reinterpret_cast<int4*>(smem + kFwdPairCap * 128);
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6, h = lane & 1;
  // the zero row (window row kFwdPairWinRows, beyond every window): skipped points' corners in the LDS-only gather
  if (tid < 64) reinterpret_cast<f4*>(smem + kFwdPairWinRows * 128)[tid] = f4{0.f, 0.f, 0.f, 0.f};
  const int ntiles = geo.nty * geo.ntx;
  int m, b;
  fwd_block(geo, M, m, b);
  const int n = b / ntiles, tile = b - n * ntiles;
  const int ty = tile / geo.ntx, tx = tile - ty * geo.ntx;
  int qy0[LT], qy1[LT], qx0[LT], qx1[LT], qc[LT + 1];
  qc[0] = 0;
#pragma unroll
  for (int l = 0; l < LT; ++l) {
    qy0[l] = tile_lo(ty, geo.H[l], geo.nty); qy1[l] = tile_lo(ty + 1, geo.H[l], geo.nty);
    qx0[l] = tile_lo(tx, geo.W[l], geo.ntx); qx1[l] = tile_lo(tx + 1, geo.W[l], geo.ntx);
    qc[l + 1] = qc[l] + (qy1[l] - qy0[l]) * (qx1[l] - qx0[l]);
  }
  const int Qt = qc[LT];
  const char* vbytes = reinterpret_cast<const char*>(value);
  const int rsb = M * D * 4;  // value row stride in bytes; value bytes < 2^31 (host check)
  unsigned chw = 16u * h;     // this lane's 16 bytes of each 32-byte piece (window and HBM rows alike)
  asm volatile("" : "+v"(chw));
  const char* pbytes = reinterpret_cast<const char*>(fe.proj);
  const char* rbytes = reinterpret_cast<const char*>(fe.ref) + static_cast<int64_t>(n) * fe.ref_bs * 4;
  const unsigned pld = static_cast<unsigned>(fe.ld) * 4u;
  // this pair's query: the tile's queries level by level, row-major in each level's rectangle; ds_read_b128 lane
  // group g of the wave ({0-3, 12-15, 20-27} + 32 (g >> 1) for even g, {4-11, 16-19, 28-31} + 32 (g >> 1) for odd)
  // takes the wave's queries 8g .. 8g + 7, quad u of the group's lanes (in lane order) queries 2u, 2u + 1
  int qi;
  {
    const int u = (lane >> 2) & 7;                             // quad within the wave's half
    const int g = ((lane >> 5) << 1) | ((0x96 >> u) & 1);      // quads 1, 2, 4, 7 are the odd groups' lanes
    qi = wid * 32 + g * 8 + (u >> 1) * 2 + ((lane >> 1) & 1);
  }
  const bool qv = qi < Qt;
  int qpos;
  {
    const int qq = min(qi, Qt - 1);
    int lq = 0;
#pragma unroll
    for (int l = 1; l < LT; ++l) lq = qq >= qc[l] ? l : lq;
    int qb = 0, qw = 1, y0 = 0, x0 = 0, W = 1, st = 0;
#pragma unroll
    for (int l = 0; l < LT; ++l)
      if (l == lq) { qb = qc[l]; qw = qx1[l] - qx0[l]; y0 = qy0[l]; x0 = qx0[l]; W = geo.W[l]; st = geo.start[l]; }
    const int rr = qq - qb;
    const int yy = static_cast<int>((static_cast<float>(rr) + 0.5f) * __builtin_amdgcn_rcpf(static_cast<float>(qw)));
    const int xx = rr - yy * qw;
    qpos = st + (y0 + yy) * W + x0 + xx;
  }
  const unsigned prow = static_cast<unsigned>(n * S + qpos) * pld;
  // softmax over the pair's L*P logits with the quad kernels' arithmetic: the exact max, then the exps summed in
  // logit order (lane h holds logits l*P + 2h, l*P + 2h + 1)
  float wa[LT][2];
  {
    const unsigned lgb = prow + static_cast<unsigned>(fe.lg0(m, M, LP) + 2 * h) * 4u;
    float mx = -INFINITY;
#pragma unroll
    for (int l = 0; l < LT; ++l) {
      const float2 t = *reinterpret_cast<const float2*>(pbytes + lgb + l * P * 4);
      wa[l][0] = t.x;
      wa[l][1] = t.y;
      mx = fmaxf(mx, t.x);
      mx = fmaxf(mx, t.y);
    }
    mx = fmaxf(mx, qpermf<0xB1>(mx));
    float sum = 0.f;
#pragma unroll
    for (int l = 0; l < LT; ++l) {
      wa[l][0] = expf(wa[l][0] - mx);
      wa[l][1] = expf(wa[l][1] - mx);
      sum += pbcast<0>(wa[l][0]);
      sum += pbcast<0>(wa[l][1]);
      sum += pbcast<1>(wa[l][0]);
      sum += pbcast<1>(wa[l][1]);
    }
    const float inv = 1.f / sum;
#pragma unroll
    for (int l = 0; l < LT; ++l) { wa[l][0] *= inv; wa[l][1] *= inv; }
  }
  const f4 z = {0.f, 0.f, 0.f, 0.f};
  f4 acc[4] = {z, z, z, z};  // channels 8k + 4h .. 8k + 4h + 3

#pragma unroll
  for (int l = 0; l < LT; ++l) {
    const int H = geo.H[l], W = geo.W[l];
    const int lbase = ((n * S + geo.start[l]) * M + m) * D * 4;
    int zq = 0;  // the level's loads after the previous level's gather (else hoisted to the start: spills)
    asm volatile("" : "+v"(zq));
    // 1. points 2h and 2h + 1 of the level: corner block (y0, x0) clamped into the level, +1 row / column inside the
    //    level (ey, ex), the four weights (x attention weight), ok; the wave's box of touched corners
    int gy[2], gx[2], gfl[2];
    float gw[2][4];
    int bmin_y = 0x7fffffff, bmax_y = -1, bmin_x = 0x7fffffff, bmax_x = -1;
    auto geometry = [&](auto pow2) {
      constexpr bool POW2 = decltype(pow2)::value;
      const float fH = static_cast<float>(H), fW = static_cast<float>(W);
      const float fHm1 = static_cast<float>(H - 1), fWm1 = static_cast<float>(W - 1);
      const float2 rf = *reinterpret_cast<const float2*>(rbytes + static_cast<unsigned>((qpos + zq) * LT + l) * 8u);
      const f4 off = *reinterpret_cast<const f4*>(pbytes + prow + static_cast<unsigned>(zq) * pld +
                                                  static_cast<unsigned>(fe.off0(m, LP) + (l * P + 2 * h) * 2) * 4u);
#pragma unroll
      for (int s = 0; s < 2; ++s) {
        const float sx = rf.x + div_norm(s ? off.z : off.x, fW, geo.invW[l], POW2);
        const float sy = rf.y + div_norm(s ? off.w : off.y, fH, geo.invH[l], POW2);
        const float hh = sy * H - 0.5f, ww = sx * W - 0.5f;
        const bool ok = qv && hh > -1.f && ww > -1.f && hh < fH && ww < fW;
        const float hs = ok ? hh : -2.f, ws = ok ? ww : -2.f;
        const float fh = floorf(hs), fw = floorf(ws);
        const float ly = hs - fh, lx = ws - fw, hy = 1.f - ly, hx = 1.f - lx;
        const bool vy0 = fh >= 0.f, vy1 = fh < fHm1, vx0 = fw >= 0.f, vx1 = fw < fWm1;
        const int y0 = static_cast<int>(__builtin_amdgcn_fmed3f(fh, 0.f, fHm1));
        const int x0 = static_cast<int>(__builtin_amdgcn_fmed3f(fw, 0.f, fWm1));
        const int ey = (vy0 && vy1) ? 1 : 0, ex = (vx0 && vx1) ? 1 : 0;
        const float a = wa[l][s];
        gw[s][0] = (vy0 && vx0) ? hy * hx * a : 0.f;
        gw[s][1] = (vy0 && vx1) ? hy * lx * a : 0.f;
        gw[s][2] = (vy1 && vx0) ? ly * hx * a : 0.f;
        gw[s][3] = (ok && vy1 && vx1) ? ly * lx * a : 0.f;  // ok: a skipped point's 0 * 0 * a could be a NaN
        gy[s] = y0;
        gx[s] = x0;
        gfl[s] = (ok ? 1 : 0) | (ey << 1) | (ex << 2);
        asm volatile("" : "+v"(gw[s][0]), "+v"(gw[s][1]), "+v"(gw[s][2]), "+v"(gw[s][3]), "+v"(gy[s]), "+v"(gx[s]),
                     "+v"(gfl[s]));
        if (ok) {
          bmin_y = min(bmin_y, y0); bmax_y = max(bmax_y, y0 + ey);
          bmin_x = min(bmin_x, x0); bmax_x = max(bmax_x, x0 + ex);
        }
      }
    };
    if (((W & (W - 1)) | (H & (H - 1))) == 0) geometry(std::true_type{});
    else geometry(std::false_type{});
    bmin_y = wave_minmax<false>(bmin_y); bmax_y = wave_minmax<true>(bmax_y);
    bmin_x = wave_minmax<false>(bmin_x); bmax_x = wave_minmax<true>(bmax_x);
    if (lane == 0) bbw[l * NW + wid] = make_int4(bmin_y, bmax_y, bmin_x, bmax_x);
    __syncthreads();  // the boxes are in; every wave is done reading the previous level's window
    // 2. the window: the box clipped to the tile +- halo, the halo shrinking until the rows fit (uniform)
    int by0 = 0x7fffffff, by1 = -1, bx0 = 0x7fffffff, bx1 = -1;
#pragma unroll
    for (int w = 0; w < NW; ++w) {
      const int4 t = bbw[l * NW + w];
      by0 = min(by0, t.x); by1 = max(by1, t.y); bx0 = min(bx0, t.z); bx1 = max(bx1, t.w);
    }
    by0 = __builtin_amdgcn_readfirstlane(by0); by1 = __builtin_amdgcn_readfirstlane(by1);
    bx0 = __builtin_amdgcn_readfirstlane(bx0); bx1 = __builtin_amdgcn_readfirstlane(bx1);
    int wy0 = 0, wy1 = -1, wx0 = 0, wx1 = -1;
    for (int halo = geo.max_halo; halo >= 0 && by1 >= 0; --halo) {
      wy0 = max(by0, qy0[l] - halo); wy1 = min(by1, qy1[l] - 1 + halo);
      wx0 = max(bx0, qx0[l] - halo); wx1 = min(bx1, qx1[l] - 1 + halo);
      if (wy1 < wy0 || wx1 < wx0) { wy1 = wy0 - 1; break; }
      if ((wy1 - wy0 + 1) * (wx1 - wx0 + 1) <= cap) break;
      if (halo == 0) wy1 = wy0 - 1;
    }
    const int wh = wy1 >= wy0 ? wy1 - wy0 + 1 : 0, wwid = wh > 0 ? wx1 - wx0 + 1 : 0;
    const int rows = wh * wwid;
    {
      const float iww = wwid > 0 ? 1.f / static_cast<float>(wwid) : 0.f;
      const int nblk = (rows + 7) >> 3;
      for (int blk = wid; blk < nblk; blk += NW) {
        // lane l fills 16 bytes of line l >> 4: row blk * 8 + ((l >> 1) & 7), 16-byte chunk 2 (l >> 4) + (l & 1)
        const int r = min(blk * 8 + ((lane >> 1) & 7), rows - 1);
        const int yy = static_cast<int>((static_cast<float>(r) + 0.5f) * iww), xx = r - yy * wwid;
        const unsigned c = static_cast<unsigned>(((lane >> 4) << 1) | (lane & 1));
        const unsigned goff = static_cast<unsigned>(mad_u24((wy0 + yy) * W + wx0 + xx, rsb, lbase)) + 16u * c;
        __builtin_amdgcn_global_load_lds(reinterpret_cast<const void*>(vbytes + goff),
                                         (__attribute__((address_space(3))) void*)(smem + blk * 1024), 16, 0, 0);
      }
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }
    __syncthreads();  // the window is in LDS
    // 3. gather: the pair's four points in order, lane h reading its 16 bytes of each 32-byte piece of a corner row
    const auto* win = (const __attribute__((address_space(3))) unsigned char*)smem;
    auto lds4 = [&](unsigned o) { return *(const __attribute__((address_space(3))) f4*)(win + o); };
    int md[2];
    unsigned a1[2], a2[2], a3[2], a4[2];
#pragma unroll
    for (int s = 0; s < 2; ++s) {
      const int fl = gfl[s], y0 = gy[s], x0 = gx[s];
      const int ey = (fl >> 1) & 1, ex = (fl >> 2) & 1;
      const bool ok = fl & 1;
      const bool inwin = ok && y0 >= wy0 && y0 + ey <= wy1 && x0 >= wx0 && x0 + ex <= wx1;
      md[s] = ok ? (inwin ? 1 : 2) : 0;
      // window form (a skipped point's corners on the zero row) or, out of the window, HBM byte offsets
      const int q1 = inwin ? (y0 - wy0) * wwid + (x0 - wx0) : kFwdPairWinRows;
      const int qx = inwin ? ex : 0, q3 = q1 + (inwin && ey ? wwid : 0);
      const unsigned g1 = static_cast<unsigned>(mad_u24(mad_u24(y0, W, x0), rsb, lbase));
      const unsigned dx = ex ? rsb : 0u, dy = ey ? static_cast<unsigned>(W * rsb) : 0u;
      const bool hbm = md[s] == 2;
      a1[s] = hbm ? g1 : pwin_row(q1);
      a2[s] = hbm ? g1 + dx : pwin_row(q1 + qx);
      a3[s] = hbm ? g1 + dy : pwin_row(q3);
      a4[s] = hbm ? g1 + dy + dx : pwin_row(q3 + qx);
    }
    auto fmas = [&](const f4* v, float u1, float u2, float u3, float u4) {
#pragma unroll
      for (int k = 0; k < 4; ++k) acc[k] += u1 * v[k];
#pragma unroll
      for (int k = 0; k < 4; ++k) acc[k] += u2 * v[4 + k];
#pragma unroll
      for (int k = 0; k < 4; ++k) acc[k] += u3 * v[8 + k];
#pragma unroll
      for (int k = 0; k < 4; ++k) acc[k] += u4 * v[12 + k];
    };
    if (!__any(md[0] == 2 || md[1] == 2)) {
      // window rows only (the common case): no mode broadcast or branch per point
      auto point = [&](auto pp) {
        constexpr int p = decltype(pp)::value, HS = p >> 1, SL = p & 1;
        unsigned b1, b2, b3, b4;
        dpp_add4p<HS>(b1, b2, b3, b4, a1[SL], a2[SL], a3[SL], a4[SL], chw);
        f4 v[16];
#pragma unroll
        for (int k = 0; k < 4; ++k) {
          v[k] = lds4(b1 + 256u * k); v[4 + k] = lds4(b2 + 256u * k);
          v[8 + k] = lds4(b3 + 256u * k); v[12 + k] = lds4(b4 + 256u * k);
        }
        fmas(v, pbcast<HS>(gw[SL][0]), pbcast<HS>(gw[SL][1]), pbcast<HS>(gw[SL][2]), pbcast<HS>(gw[SL][3]));
      };
      point(std::integral_constant<int, 0>{});
      point(std::integral_constant<int, 1>{});
      point(std::integral_constant<int, 2>{});
      point(std::integral_constant<int, 3>{});
    } else {
      auto point = [&](auto pp) {
        constexpr int p = decltype(pp)::value, HS = p >> 1, SL = p & 1;
        const int mq = pbcasti<HS>(md[SL]);
        unsigned b1, b2, b3, b4;
        dpp_add4p<HS>(b1, b2, b3, b4, a1[SL], a2[SL], a3[SL], a4[SL], chw);
        const float u1 = pbcast<HS>(gw[SL][0]), u2 = pbcast<HS>(gw[SL][1]);
        const float u3 = pbcast<HS>(gw[SL][2]), u4 = pbcast<HS>(gw[SL][3]);
        f4 v[16];
        if (mq == 2) {
#pragma unroll
          for (int k = 0; k < 4; ++k) {
            v[k] = ldb4(vbytes, b1 + 32u * k); v[4 + k] = ldb4(vbytes, b2 + 32u * k);
            v[8 + k] = ldb4(vbytes, b3 + 32u * k); v[12 + k] = ldb4(vbytes, b4 + 32u * k);
          }
          fmas(v, u1, u2, u3, u4);
        } else if (mq == 1) {
#pragma unroll
          for (int k = 0; k < 4; ++k) {
            v[k] = lds4(b1 + 256u * k); v[4 + k] = lds4(b2 + 256u * k);
            v[8 + k] = lds4(b3 + 256u * k); v[12 + k] = lds4(b4 + 256u * k);
          }
          fmas(v, u1, u2, u3, u4);
        }
      };
      point(std::integral_constant<int, 0>{});
      point(std::integral_constant<int, 1>{});
      point(std::integral_constant<int, 2>{});
      point(std::integral_constant<int, 3>{});
    }
  }
  if (qv) {
    char* o = reinterpret_cast<char*>(out) + (static_cast<unsigned>((n * S + qpos) * M + m) * 128u + 16u * h);
#pragma unroll
    for (int k = 0; k < 4; ++k) *reinterpret_cast<f4*>(o + 32 * k) = acc[k];
  }
}

// ------------------------------------------------------------------------------------------------
// Host side
// ------------------------------------------------------------------------------------------------

struct Dims {
  int N, S, M, D, L, Lq, P;
  int64_t npairs() const { return static_cast<int64_t>(N) * Lq * M; }
};

int check_dims(const char* fn, const void* value, const void* shapes, const void* lsi, const void* loc,
               const void* attn, const Dims& d, int im2col_step) {
  if (!value || !shapes || !lsi || !loc || !attn)
    return m2f::fail(M2F_EINVAL, "%s: null input pointer", fn);
  if (d.N <= 0 || d.S <= 0 || d.M <= 0 || d.D <= 0 || d.L <= 0 || d.Lq <= 0 || d.P <= 0)
    return m2f::fail(M2F_EINVAL, "%s: non-positive size (N=%d S=%d M=%d D=%d L=%d Lq=%d P=%d)", fn, d.N,
                     d.S, d.M, d.D, d.L, d.Lq, d.P);
  if (im2col_step <= 0) return m2f::fail(M2F_EINVAL, "%s: im2col_step must be positive", fn);
  const int step = std::min(d.N, im2col_step);
  if (d.N % step != 0)
    return m2f::fail(M2F_EINVAL, "%s: batch(%d) must divide im2col_step(%d)", fn, d.N, step);
  return M2F_OK;
}

bool fast_f32_ok(const Dims& d, const void* value, const void* loc, const void* out4) {
  const bool dims = (d.D == 16 || d.D == 32 || d.D == 64) && d.L <= kMaxLevels;
  return dims && m2f::aligned(value, 16) && m2f::aligned(loc, 8) && m2f::aligned(out4, 16);
}

template <int D>
void launch_fwd_vec(const float* value, const int64_t* shapes, const int64_t* lsi, const float* loc,
                    const float* attn, const Dims& d, float* out, hipStream_t st) {
  constexpr int G = D / 4;
  const unsigned grid = m2f::ceil_div(d.npairs(), 256 / G);
  if (d.P == 4)
    msda_fwd_f32_vec<D, 4><<<grid, 256, 0, st>>>(value, shapes, lsi, loc, attn, d.npairs(), d.S, d.M, d.L,
                                                  d.Lq, d.P, out);
  else
    msda_fwd_f32_vec<D, 0><<<grid, 256, 0, st>>>(value, shapes, lsi, loc, attn, d.npairs(), d.S, d.M, d.L,
                                                  d.Lq, d.P, out);
}

template <int D>
void launch_bwd_vec(const float* value, const int64_t* shapes, const int64_t* lsi, const float* loc,
                    const float* attn, const float* gout, const Dims& d, float* gv, float* gl, float* ga,
                    hipStream_t st) {
  constexpr int G = D / 4;
  const unsigned grid = m2f::ceil_div(d.npairs(), 256 / G);
  if (d.P == 4)
    msda_bwd_f32_vec<D, 4><<<grid, 256, 0, st>>>(value, shapes, lsi, loc, attn, gout, d.npairs(), d.S, d.M,
                                                  d.L, d.Lq, d.P, gv, gl, ga);
  else
    msda_bwd_f32_vec<D, 0><<<grid, 256, 0, st>>>(value, shapes, lsi, loc, attn, gout, d.npairs(), d.S, d.M,
                                                  d.L, d.Lq, d.P, gv, gl, ga);
}

bool make_fwd_lds_geom(const Dims& d, int proj_ld, const TileGeom& base, TileGeom& geo, size_t& lds,
                       bool pair = false);
bool launch_fwd_lds_unfused(const float* value, const float* loc, const float* attn, const Dims& d,
                            const int64_t* host_shapes, float* out, hipStream_t st);

template <typename T>
int fwd_impl(const char* fn, const T* value, const int64_t* shapes, const int64_t* lsi, const T* loc,
             const T* attn, const Dims& d, int im2col_step, T* out, hipStream_t st,
             const int64_t* host_shapes = nullptr) {
  int rc = check_dims(fn, value, shapes, lsi, loc, attn, d, im2col_step);
  if (rc) return rc;
  if (!out) return m2f::fail(M2F_EINVAL, "%s: null output", fn);
  bool done = false;
  if constexpr (std::is_same<T, float>::value) {
    if (fast_f32_ok(d, value, loc, out)) {
      if (launch_fwd_lds_unfused(value, loc, attn, d, host_shapes, out, st)) {
      } else if (d.D == 16) launch_fwd_vec<16>(value, shapes, lsi, loc, attn, d, out, st);
      else if (d.D == 32 && d.P == 4 && m2f::option(m2f::kOptMsdaFwdQuad, 1) != 0 &&
               static_cast<int64_t>(d.N) * d.S * d.M * d.D * 4 < (int64_t{1} << 31))
        msda_fwd_f32_q4<<<m2f::ceil_div(d.npairs(), 64), 256, 0, st>>>(value, shapes, lsi, loc, attn, d.npairs(), d.S,
                                                                        d.M, d.L, d.Lq, out);
      else if (d.D == 32) launch_fwd_vec<32>(value, shapes, lsi, loc, attn, d, out, st);
      else launch_fwd_vec<64>(value, shapes, lsi, loc, attn, d, out, st);
      done = true;
    }
  }
  if (!done) {
    const int64_t total = d.npairs() * d.D;
    const unsigned grid = static_cast<unsigned>(std::min<int64_t>((total + 255) / 256, 256 * 64));
    msda_fwd_generic<T><<<grid, 256, 0, st>>>(value, shapes, lsi, loc, attn, total, d.S, d.M, d.D, d.L, d.Lq,
                                               d.P, out);
  }
  return m2f::check_launch(fn);
}

// Tile geometry for the tiled backward; false when the configuration does not qualify (then the
// caller uses the untiled kernels).  Lq == S: the queries are the flattened pyramid.
// Options (m2f_set_option):
//   msda_threads (1024; 512 in the deterministic mode): workgroup size, 512 (two workgroups per CU) or 1024 (one);
//   msda_tile / msda_tile_w (12 / 12 at 512 threads, 16 / 16 at 1024): tile on the finest level;
//   msda_halo (8 at 512 threads, 12 at 1024): window halo;  msda_win_rows (cells per workgroup; the halo shrinks until the
//   window fits).  Geometry only: every setting computes the same gradients (tests sweep them).
bool make_tile_geom(const Dims& d, const int64_t* host_shapes, TileGeom& geo, size_t& lds, int& threads) {
  if (!host_shapes || d.D != 32 || d.P != 4 || d.Lq != d.S || d.L > kTileMaxL) return false;
  if (static_cast<int64_t>(d.N) * d.S * d.M * d.D * 4 >= (int64_t{1} << 31)) return false;  // 32-bit byte offsets
  // the op-level (unfused) kernels address loc (8 B per sample) and grad_attn / grad_loc in 32 bits
  if (static_cast<int64_t>(d.N) * d.Lq * d.M * d.L * d.P * 8 >= (int64_t{1} << 31)) return false;
  geo = TileGeom{};
  geo.L = d.L;
  int64_t total = 0;
  int fi = 0;
  for (int l = 0; l < d.L; ++l) {
    geo.H[l] = static_cast<int>(host_shapes[2 * l]);
    geo.W[l] = static_cast<int>(host_shapes[2 * l + 1]);
    if (geo.H[l] <= 0 || geo.W[l] <= 0) return false;
    // phase 2 forms corner offsets (y0 * W + x0) * rs with 24-bit multiplies (__umul24): a level of 2^24 or
    // more pixels would silently wrap, so such shapes take the untiled kernels
    if (static_cast<int64_t>(geo.H[l]) * geo.W[l] >= (int64_t{1} << 24)) return false;
    // the descriptors pack each floor + 2 (-2 .. H - 1) in 16 bits
    if (geo.H[l] > 65533 || geo.W[l] > 65533) return false;
    geo.start[l] = static_cast<int>(total);
    geo.invW[l] = 1.f / static_cast<float>(geo.W[l]);
    geo.invH[l] = 1.f / static_cast<float>(geo.H[l]);
    total += static_cast<int64_t>(geo.H[l]) * geo.W[l];
    if (static_cast<int64_t>(geo.H[l]) * geo.W[l] > static_cast<int64_t>(geo.H[fi]) * geo.W[fi]) fi = l;
  }
  if (total != d.S) return false;
  // 1024 threads with 16x16 tiles and a halo of 12 (one workgroup per CU): at config 2 1.707 ms with near-init
  // sampling against 1.697 for 512 threads / 12x12 / halo 8 (two per CU), and 2.43 against 4.51 ms with N(0, 4 px)
  // offsets, where the larger tiles flush fewer window rows per owned row and the halo keeps samples out of the
  // direct atomics (profiles/r04_i*_mb.txt).  The deterministic mode keeps 512 / 12x12 / 8 (2.74 vs 3.55 ms).
  const bool det = m2f::option(m2f::kOptMsdaBwdDet, 0) != 0;
  // four levels: 512-thread workgroups only (the L = 4 body needs more than the 128 VGPRs of a 1024-thread one)
  const int first = d.L == 4 ? 512 : m2f::option(m2f::kOptMsdaThreads, det ? 512 : 1024) >= 1024 ? 1024 : 512;
  geo.ratio23 = std::max(1, m2f::option(m2f::kOptMsdaBwdRatio, 1));
  geo.rowsort = m2f::option(m2f::kOptMsdaBwdRowSort, 1) != 0 ? 1 : 0;
  geo.walk4 = m2f::option(m2f::kOptMsdaBwdWalk4, 1) != 0 ? 1 : 0;
  const TileGeom base = geo;
  // a default 1024-thread geometry whose LDS does not fit (e.g. four levels: 16 samples per query) falls back to
  // the 512-thread one; an explicit msda_threads does not
  for (int attempt = 0; attempt < 2; ++attempt) {
    if (attempt == 1 && (first == 512 || m2f::option_raw(m2f::kOptMsdaThreads) >= 0)) break;
    threads = attempt == 0 ? first : 512;
    geo = base;
    const int tile_h = std::max(1, m2f::option(m2f::kOptMsdaTile, threads == 1024 ? 16 : 12));
    const int tile_w = std::max(1, m2f::option(m2f::kOptMsdaTileW, tile_h));
    geo.nty = (geo.H[fi] + tile_h - 1) / tile_h;
    geo.ntx = (geo.W[fi] + tile_w - 1) / tile_w;
    geo.max_halo = std::max(0, m2f::option(m2f::kOptMsdaHalo, threads == 1024 ? 12 : 8));
    // cells of the largest window any workgroup can choose (tile + 2 halo + 1 per axis, clipped to the level),
    // unless a smaller budget is asked for; it must hold every level's share of one tile at halo 0 (tiles
    // span at most ceil(n / nt) pixels per axis, tile_lo) plus the extra cell row / column
    int own = 0, qt = 0, full = 0;
    for (int l = 0; l < d.L; ++l) {
      const int th = (geo.H[l] + geo.nty - 1) / geo.nty, tw = (geo.W[l] + geo.ntx - 1) / geo.ntx;
      own += (std::min(geo.H[l], th + 1) + 1) * (std::min(geo.W[l], tw + 1) + 1);  // clipped like `full`
      full += (std::min(geo.H[l], th + 2 * geo.max_halo) + 1) * (std::min(geo.W[l], tw + 2 * geo.max_halo) + 1);
      qt += th * tw;
    }
    geo.max_rows = m2f::option(m2f::kOptMsdaWinRows, full);
    geo.max_qt = qt;
    const int lp = d.L * d.P;
    // phase 3's 32-bit slots hold the g-row byte offset 128 * qs (qs <= qt: the zero row) in their low 16 bits
    if (own > geo.max_rows || static_cast<int64_t>(qt) * lp >= 0xffff || qt > 511) continue;
    if (static_cast<int64_t>(qt) * lp > kSortSamples) continue;
    const size_t ns = static_cast<size_t>(qt) * lp;
    lds = ((static_cast<size_t>(qt) + 1) * 32 + ns * 4 + (threads / 64) * kStageFloats) * 4 +
          ((static_cast<size_t>(geo.max_rows) + 1 + 3) & ~static_cast<size_t>(3)) * 4 +
          (((ns + 31) / 32 + 3) & ~static_cast<size_t>(3)) * 4 + (ns + 8) * 4 + static_cast<size_t>(qt) * 4;
    if (lds <= 156 * 1024) return true;
  }
  return false;
}

// Deterministic-mode buffers (msda_bwd_det): the int64 accumulator of grad_value and the scale words.
struct DetBufs {
  unsigned long long* acc = nullptr;
  unsigned* scale = nullptr;  // [max |g| bits, non-finite flag]
};

template <int LT, bool FUSED, int TPB>
int launch_tiled_t(const float* value, const float* loc, const float* attn, const FrontEnd& fe, const float* gout,
                   const TileGeom& geo, size_t lds, const Dims& d, float* gv, float* gl, float* ga, const DetBufs& det,
                   hipStream_t st) {
  const dim3 grid(geo.nty * geo.ntx * d.M * d.N);
  const char* fn = "msda tiled backward";
  constexpr int kLds = 160 * 1024 - 1024;   // the static TileState (< 1 KB) shares the 160 KB
  if (det.acc) {
    auto* k = &msda_bwd_f32_tiled<LT, FUSED, TPB, true, true>;
    if (int rc = m2f::set_max_lds(reinterpret_cast<const void*>(k), kLds, fn)) return rc;
    k<<<grid, TPB, lds, st>>>(value, loc, attn, fe, gout, geo, d.S, d.M, gv, gl, ga, det.acc, det.scale, nullptr);
  } else if (m2f::option(m2f::kOptMsdaBwdOverlap, 1) != 0) {
    auto* k = &msda_bwd_f32_tiled<LT, FUSED, TPB, true>;
    if (int rc = m2f::set_max_lds(reinterpret_cast<const void*>(k), kLds, fn)) return rc;
    k<<<grid, TPB, lds, st>>>(value, loc, attn, fe, gout, geo, d.S, d.M, gv, gl, ga, nullptr, nullptr, nullptr);
  } else {
    auto* k = &msda_bwd_f32_tiled<LT, FUSED, TPB, false>;
    if (int rc = m2f::set_max_lds(reinterpret_cast<const void*>(k), kLds, fn)) return rc;
    k<<<grid, TPB, lds, st>>>(value, loc, attn, fe, gout, geo, d.S, d.M, gv, gl, ga, nullptr, nullptr, nullptr);
  }
  return M2F_OK;
}

template <int LT, bool FUSED>
int launch_tiled(const float* value, const float* loc, const float* attn, const FrontEnd& fe, const float* gout,
                 const TileGeom& geo, size_t lds, int threads, const Dims& d, float* gv, float* gl, float* ga,
                 const DetBufs& det, hipStream_t st) {
  if constexpr (LT < 4) {
    if (threads == 1024) return launch_tiled_t<LT, FUSED, 1024>(value, loc, attn, fe, gout, geo, lds, d, gv, gl, ga, det, st);
  }
  return launch_tiled_t<LT, FUSED, 512>(value, loc, attn, fe, gout, geo, lds, d, gv, gl, ga, det, st);
}

// M2F status of the launch (an LDS-attribute failure returns before the kernel is launched)
template <bool FUSED>
int launch_tiled_levels(const float* value, const float* loc, const float* attn, const FrontEnd& fe, const float* gout,
                        const TileGeom& geo, size_t lds, int threads, const Dims& d, float* gv, float* gl, float* ga,
                        hipStream_t st, const DetBufs& det = DetBufs{}) {
  switch (d.L) {
    case 1: return launch_tiled<1, FUSED>(value, loc, attn, fe, gout, geo, lds, threads, d, gv, gl, ga, det, st);
    case 2: return launch_tiled<2, FUSED>(value, loc, attn, fe, gout, geo, lds, threads, d, gv, gl, ga, det, st);
    case 3: return launch_tiled<3, FUSED>(value, loc, attn, fe, gout, geo, lds, threads, d, gv, gl, ga, det, st);
    default: return launch_tiled<4, FUSED>(value, loc, attn, fe, gout, geo, lds, threads, d, gv, gl, ga, det, st);
  }
}

// -1: the tiled kernel does not apply (the caller takes another kernel); else the M2F status of its launch
int launch_bwd_tiled(const float* value, const float* loc, const float* attn, const float* gout, const Dims& d,
                     const int64_t* host_shapes, float* gv, float* gl, float* ga, hipStream_t st) {
  if (m2f::option(m2f::kOptMsdaBwdTiled, 1) == 0) return -1;
  TileGeom geo;
  size_t lds;
  int threads;
  if (!make_tile_geom(d, host_shapes, geo, lds, threads)) return -1;
  return launch_tiled_levels<false>(value, loc, attn, FrontEnd{}, gout, geo, lds, threads, d, gv, gl, ga, st);
}

template <typename T>
int bwd_impl(const char* fn, const T* value, const int64_t* shapes, const int64_t* lsi, const T* loc,
             const T* attn, const T* gout, const Dims& d, int im2col_step, const int64_t* host_shapes, T* gv,
             T* gl, T* ga, hipStream_t st) {
  int rc = check_dims(fn, value, shapes, lsi, loc, attn, d, im2col_step);
  if (rc) return rc;
  if (!gout || !gv || !gl || !ga) return m2f::fail(M2F_EINVAL, "%s: null gradient pointer", fn);
  const size_t gv_bytes = static_cast<size_t>(d.N) * d.S * d.M * d.D * sizeof(T);
  hipError_t e = m2f::zero_async(gv, gv_bytes, st);
  if (e != hipSuccess) return m2f::fail(M2F_ELAUNCH, "%s: memset grad_value: %s", fn, hipGetErrorString(e));
  bool done = false;
  if constexpr (std::is_same<T, float>::value) {
    if (fast_f32_ok(d, value, loc, gout) && m2f::aligned(gv, 16) && m2f::aligned(gl, 8)) {
      const int trc = launch_bwd_tiled(value, loc, attn, gout, d, host_shapes, gv, gl, ga, st);
      if (trc > 0) return trc;
      if (trc == 0) done = true;
      else if (d.D == 16) launch_bwd_vec<16>(value, shapes, lsi, loc, attn, gout, d, gv, gl, ga, st);
      else if (d.D == 32) launch_bwd_vec<32>(value, shapes, lsi, loc, attn, gout, d, gv, gl, ga, st);
      else launch_bwd_vec<64>(value, shapes, lsi, loc, attn, gout, d, gv, gl, ga, st);
      done = true;
    }
  } else {
    (void)host_shapes;
  }
  if (!done) {
    const int64_t npairs = d.npairs();
    if (npairs > 0x7fffffffLL) return m2f::fail(M2F_EUNSUPPORTED, "%s: too many (n,q,m) pairs", fn);
    if (d.D <= 64)
      msda_bwd_generic<T, 64><<<static_cast<unsigned>(npairs), 64, 0, st>>>(
          value, shapes, lsi, loc, attn, gout, d.S, d.M, d.D, d.L, d.Lq, d.P, gv, gl, ga);
    else
      msda_bwd_generic<T, 256><<<static_cast<unsigned>(npairs), 256, 0, st>>>(
          value, shapes, lsi, loc, attn, gout, d.S, d.M, d.D, d.L, d.Lq, d.P, gv, gl, ga);
  }
  return m2f::check_launch(fn);
}

}  // namespace

extern "C" int m2f_msda_fwd_f32(const float* value, const int64_t* spatial_shapes, const int64_t* level_start_index,
                                const float* sampling_loc, const float* attn_weight, int batch, int spatial_size,
                                int num_heads, int channels, int num_levels, int num_query, int num_point,
                                int im2col_step, const int64_t* host_spatial_shapes, float* output, void* stream) {
  const Dims d{batch, spatial_size, num_heads, channels, num_levels, num_query, num_point};
  return fwd_impl<float>("m2f_msda_fwd_f32", value, spatial_shapes, level_start_index, sampling_loc, attn_weight,
                         d, im2col_step, output, static_cast<hipStream_t>(stream), host_spatial_shapes);
}

extern "C" int m2f_msda_fwd_f64(const double* value, const int64_t* spatial_shapes,
                                const int64_t* level_start_index, const double* sampling_loc,
                                const double* attn_weight, int batch, int spatial_size, int num_heads, int channels,
                                int num_levels, int num_query, int num_point, int im2col_step,
                                const int64_t* host_spatial_shapes, double* output, void* stream) {
  (void)host_spatial_shapes;
  const Dims d{batch, spatial_size, num_heads, channels, num_levels, num_query, num_point};
  return fwd_impl<double>("m2f_msda_fwd_f64", value, spatial_shapes, level_start_index, sampling_loc,
                          attn_weight, d, im2col_step, output, static_cast<hipStream_t>(stream));
}

extern "C" int m2f_msda_bwd_f32(const float* value, const int64_t* spatial_shapes, const int64_t* level_start_index,
                                const float* sampling_loc, const float* attn_weight, const float* grad_output,
                                int batch, int spatial_size, int num_heads, int channels, int num_levels,
                                int num_query, int num_point, int im2col_step, const int64_t* host_spatial_shapes,
                                float* grad_value, float* grad_sampling_loc, float* grad_attn_weight,
                                void* stream) {
  const Dims d{batch, spatial_size, num_heads, channels, num_levels, num_query, num_point};
  return bwd_impl<float>("m2f_msda_bwd_f32", value, spatial_shapes, level_start_index, sampling_loc, attn_weight,
                         grad_output, d, im2col_step, host_spatial_shapes, grad_value, grad_sampling_loc,
                         grad_attn_weight, static_cast<hipStream_t>(stream));
}

extern "C" int m2f_msda_bwd_f64(const double* value, const int64_t* spatial_shapes,
                                const int64_t* level_start_index, const double* sampling_loc,
                                const double* attn_weight, const double* grad_output, int batch, int spatial_size,
                                int num_heads, int channels, int num_levels, int num_query, int num_point,
                                int im2col_step, const int64_t* host_spatial_shapes, double* grad_value,
                                double* grad_sampling_loc, double* grad_attn_weight, void* stream) {
  const Dims d{batch, spatial_size, num_heads, channels, num_levels, num_query, num_point};
  return bwd_impl<double>("m2f_msda_bwd_f64", value, spatial_shapes, level_start_index, sampling_loc,
                          attn_weight, grad_output, d, im2col_step, host_spatial_shapes, grad_value,
                          grad_sampling_loc, grad_attn_weight, static_cast<hipStream_t>(stream));
}

// ------------------------------------------------------------------------------------------------
// Fused front end C ABI
// ------------------------------------------------------------------------------------------------
namespace {

int64_t det_workspace_bytes(const Dims& d) {
  return static_cast<int64_t>(d.N) * d.S * d.M * d.D * 8 + 16;  // int64 grad_value accumulator + scale words
}

int fused_check(const char* fn, const float* value, const float* proj, int ld, const float* ref,
                const int64_t* host_shapes, const Dims& d, TileGeom& geo) {
  if (!value || !proj || !ref || !host_shapes) return m2f::fail(M2F_EINVAL, "%s: null pointer", fn);
  if (d.N <= 0 || d.S <= 0 || d.M <= 0 || d.Lq <= 0) return m2f::fail(M2F_EINVAL, "%s: non-positive size", fn);
  if (d.D != 32 || d.P != 4 || d.L < 1 || d.L > kTileMaxL)
    return m2f::fail(M2F_EUNSUPPORTED, "%s: needs channels 32, points 4, 1..4 levels (got D=%d P=%d L=%d)", fn,
                     d.D, d.P, d.L);
  if (ld < d.M * d.L * d.P * 3 || (ld & 1))
    return m2f::fail(M2F_EINVAL, "%s: projection row stride %d (need even, >= %d)", fn, ld, d.M * d.L * d.P * 3);
  if (!m2f::aligned(value, 16) || !m2f::aligned(proj, 8) || !m2f::aligned(ref, 8))
    return m2f::fail(M2F_EINVAL, "%s: misaligned input", fn);
  geo = TileGeom{};
  geo.L = d.L;
  int64_t total = 0;
  for (int l = 0; l < d.L; ++l) {
    geo.H[l] = static_cast<int>(host_shapes[2 * l]);
    geo.W[l] = static_cast<int>(host_shapes[2 * l + 1]);
    if (geo.H[l] <= 0 || geo.W[l] <= 0) return m2f::fail(M2F_EINVAL, "%s: bad level shape", fn);
    geo.start[l] = static_cast<int>(total);
    geo.invW[l] = 1.f / static_cast<float>(geo.W[l]);
    geo.invH[l] = 1.f / static_cast<float>(geo.H[l]);
    total += static_cast<int64_t>(geo.H[l]) * geo.W[l];
  }
  if (total != d.S) return m2f::fail(M2F_EINVAL, "%s: sum of H*W (%lld) != spatial_size (%d)", fn,
                                     static_cast<long long>(total), d.S);
  return M2F_OK;
}

// Geometry of the LDS-window forward; false when the configuration does not qualify (then the quad kernel runs).
// Options: msda_fwd_tile / msda_fwd_tile_w (8 / 16): tile rows / columns on the finest level; msda_fwd_cap (416):
// window rows (three workgroups per CU at 52 KB); msda_fwd_halo (8): window halo.  Partition only: every setting
// computes the same output.
bool make_fwd_lds_geom(const Dims& d, int proj_ld, const TileGeom& base, TileGeom& geo, size_t& lds, bool pair) {
  if (d.D != 32 || d.P != 4 || d.Lq != d.S || d.L > kTileMaxL) return false;
  // 32-bit byte offsets into value / out, proj and one image's reference points
  if (static_cast<int64_t>(d.N) * d.S * d.M * d.D * 4 >= (int64_t{1} << 31)) return false;
  if (static_cast<int64_t>(d.N) * d.S * proj_ld * 4 >= (int64_t{1} << 31)) return false;
  if (static_cast<int64_t>(d.S) * d.L * 8 >= (int64_t{1} << 31)) return false;
  geo = base;
  int fi = 0;
  for (int l = 0; l < d.L; ++l) {
    if (static_cast<int64_t>(geo.H[l]) * geo.W[l] >= (int64_t{1} << 24)) return false;  // 24-bit multiplies
    if (static_cast<int64_t>(geo.H[l]) * geo.W[l] > static_cast<int64_t>(geo.H[fi]) * geo.W[fi]) fi = l;
  }
  const int th = std::max(1, m2f::option(m2f::kOptMsdaFwdTile, 8));
  const int tw = std::max(1, m2f::option(m2f::kOptMsdaFwdTileW, pair ? 12 : 16));
  geo.nty = (geo.H[fi] + th - 1) / th;
  geo.ntx = (geo.W[fi] + tw - 1) / tw;
  geo.max_halo = std::max(0, m2f::option(m2f::kOptMsdaFwdHalo, 8));
  const int win_rows = pair ? kFwdPairWinRows : kFwdWinRows;
  const int cap = std::min(m2f::option(m2f::kOptMsdaFwdCap, win_rows), win_rows) & ~7;
  int qt = 0, own = 0;
  for (int l = 0; l < d.L; ++l) {
    const int h = (geo.H[l] + geo.nty - 1) / geo.nty, w = (geo.W[l] + geo.ntx - 1) / geo.ntx;
    qt += h * w;
    own = std::max(own, std::min(h + 1, geo.H[l]) * std::min(w + 1, geo.W[l]));
  }
  if (qt > (pair ? kFwdPairQueries : kFwdLdsRounds * (kFwdLdsThreads / 4)) || cap < own) return false;
  geo.max_rows = cap;
  geo.max_qt = qt;
  geo.xcdmap = m2f::option(m2f::kOptMsdaFwdXcd, 0) != 0 &&
               (static_cast<int64_t>(d.N) * geo.nty * geo.ntx) % 8 == 0 ? 1 : 0;
  lds = 0;  // static
  return true;
}

// The reference op's forward (materialised loc / attn) on the LDS-window kernel: encoder layout with host shapes,
// the options that select the windowed forward, and every byte offset under 2^31; false otherwise.
bool launch_fwd_lds_unfused(const float* value, const float* loc, const float* attn, const Dims& d,
                            const int64_t* host_shapes, float* out, hipStream_t st) {
  if (!host_shapes || d.D != 32 || d.P != 4 || d.Lq != d.S || d.L < 1 || d.L > kTileMaxL) return false;
  if (m2f::option(m2f::kOptMsdaFwdLds, 1) == 0 || m2f::option(m2f::kOptMsdaFwdQuad, 1) == 0 ||
      m2f::option(m2f::kOptMsdaFwdTiled, 1) == 0)
    return false;
  if (!m2f::aligned(loc, 8) || static_cast<int64_t>(d.N) * d.S * d.M * d.L * d.P * 8 >= (int64_t{1} << 31)) return false;
  TileGeom base{};
  base.L = d.L;
  int64_t total = 0;
  for (int l = 0; l < d.L; ++l) {
    base.H[l] = static_cast<int>(host_shapes[2 * l]);
    base.W[l] = static_cast<int>(host_shapes[2 * l + 1]);
    if (base.H[l] <= 0 || base.W[l] <= 0) return false;
    base.start[l] = static_cast<int>(total);
    base.invW[l] = 1.f / static_cast<float>(base.W[l]);
    base.invH[l] = 1.f / static_cast<float>(base.H[l]);
    total += static_cast<int64_t>(base.H[l]) * base.W[l];
  }
  if (total != d.S) return false;
  TileGeom geo;
  size_t lds = 0;
  if (!make_fwd_lds_geom(d, 0, base, geo, lds)) return false;
  const int64_t nb = static_cast<int64_t>(geo.nty) * geo.ntx * d.M * d.N;
  if (nb > 0x7fffffff) return false;
  const unsigned tg = static_cast<unsigned>(nb);
  const FrontEnd fe{};
  switch (d.L) {
    case 1: msda_fused_fwd_lds<1, false><<<tg, kFwdLdsThreads, lds, st>>>(value, fe, geo, d.S, d.M, out, loc, attn); break;
    case 2: msda_fused_fwd_lds<2, false><<<tg, kFwdLdsThreads, lds, st>>>(value, fe, geo, d.S, d.M, out, loc, attn); break;
    case 3: msda_fused_fwd_lds<3, false><<<tg, kFwdLdsThreads, lds, st>>>(value, fe, geo, d.S, d.M, out, loc, attn); break;
    default: msda_fused_fwd_lds<4, false><<<tg, kFwdLdsThreads, lds, st>>>(value, fe, geo, d.S, d.M, out, loc, attn); break;
  }
  return true;
}

}  // namespace

static int fused_fwd(int hm, const char* fn, const float* value, const float* proj, int proj_ld, const float* ref,
                                      int64_t ref_batch_stride, const int64_t* host_spatial_shapes, int batch,
                                      int spatial_size, int num_heads, int channels, int num_levels,
                                      int num_query, int num_point, float* output, void* stream) {
  const Dims d{batch, spatial_size, num_heads, channels, num_levels, num_query, num_point};
  TileGeom geo;
  int rc = fused_check(fn, value, proj, proj_ld, ref, host_spatial_shapes, d, geo);
  if (rc) return rc;
  if (!output || !m2f::aligned(output, 16)) return m2f::fail(M2F_EINVAL, "%s: bad output", fn);
  const FrontEnd fe{proj, proj_ld, ref, ref_batch_stride, hm};
  hipStream_t st = static_cast<hipStream_t>(stream);
  // value and out hold N * Lq(=S) * M * 32 elements; 32-bit offsets when those fit
  const bool off32 = static_cast<int64_t>(d.N) * std::max(d.S, d.Lq) * d.M * d.D < (int64_t{1} << 31);
  // quad form: byte offsets in 32-bit int arithmetic (value bytes < 2^31)
  const bool boff31 = static_cast<int64_t>(d.N) * d.S * d.M * d.D * 4 < (int64_t{1} << 31);
  TileGeom lgeo;
  size_t llds = 0;
  if (m2f::option(m2f::kOptMsdaFwdLds, 1) != 0 && m2f::option(m2f::kOptMsdaFwdQuad, 1) != 0 &&
      m2f::option(m2f::kOptMsdaFwdTiled, 1) != 0 && m2f::option(m2f::kOptMsdaFwdPair, 0) != 0 &&
      make_fwd_lds_geom(d, proj_ld, geo, lgeo, llds, true)) {
    const int64_t nb = static_cast<int64_t>(lgeo.nty) * lgeo.ntx * d.M * d.N;
    if (nb > 0x7fffffff) return m2f::fail(M2F_EUNSUPPORTED, "%s: too many workgroups", fn);
    const unsigned tg = static_cast<unsigned>(nb);
#define M2F_FP(LT) msda_fused_fwd_pair<LT><<<tg, kFwdPairThreads, 0, st>>>(value, fe, lgeo, d.S, d.M, output)
    switch (d.L) {
      case 1: M2F_FP(1); break;
      case 2: M2F_FP(2); break;
      case 3: M2F_FP(3); break;
      default: M2F_FP(4); break;
    }
#undef M2F_FP
    return m2f::check_launch(fn);
  }
  if (m2f::option(m2f::kOptMsdaFwdLds, 1) != 0 && m2f::option(m2f::kOptMsdaFwdQuad, 1) != 0 &&
      m2f::option(m2f::kOptMsdaFwdTiled, 1) != 0 && make_fwd_lds_geom(d, proj_ld, geo, lgeo, llds)) {
    const int64_t nb = static_cast<int64_t>(lgeo.nty) * lgeo.ntx * d.M * d.N;
    if (nb > 0x7fffffff) return m2f::fail(M2F_EUNSUPPORTED, "%s: too many workgroups", fn);
    const unsigned tg = static_cast<unsigned>(nb);
#define M2F_FL(LT) msda_fused_fwd_lds<LT><<<tg, kFwdLdsThreads, llds, st>>>(value, fe, lgeo, d.S, d.M, output)
    switch (d.L) {
      case 1: M2F_FL(1); break;
      case 2: M2F_FL(2); break;
      case 3: M2F_FL(3); break;
      default: M2F_FL(4); break;
    }
#undef M2F_FL
    return m2f::check_launch(fn);
  }
  if (boff31 && d.Lq == d.S && m2f::option(m2f::kOptMsdaFwdQuad, 1) != 0 && m2f::option(m2f::kOptMsdaFwdTiled, 1) != 0) {
    int64_t T = 0;
    for (int l = 0; l < d.L; ++l) T += static_cast<int64_t>((geo.H[l] + 7) / 8) * ((geo.W[l] + 7) / 8);
    const int64_t nb = T * d.M * d.N;
    if (nb > 0x7fffffff) return m2f::fail(M2F_EUNSUPPORTED, "%s: too many workgroups", fn);
    const unsigned tg = static_cast<unsigned>(nb);
    const int pb = m2f::option(m2f::kOptMsdaFwdPb, 2);  // points per load batch (1, 2 or 4)
#define M2F_FQ(LT)                                                                                       \
  (pb == 1   ? msda_fused_fwd_q4<LT, 1><<<tg, 256, 0, st>>>(value, fe, geo, d.S, d.M, output)            \
   : pb >= 4 ? msda_fused_fwd_q4<LT, 4><<<tg, 256, 0, st>>>(value, fe, geo, d.S, d.M, output)            \
             : msda_fused_fwd_q4<LT, 2><<<tg, 256, 0, st>>>(value, fe, geo, d.S, d.M, output))
    switch (d.L) {
      case 1: M2F_FQ(1); break;
      case 2: M2F_FQ(2); break;
      case 3: M2F_FQ(3); break;
      default: M2F_FQ(4); break;
    }
#undef M2F_FQ
    return m2f::check_launch(fn);
  }
  if (m2f::option(m2f::kOptMsdaFwdTiled, 1) != 0 && d.Lq == d.S) {
    int64_t T = 0;
    for (int l = 0; l < d.L; ++l) T += static_cast<int64_t>((geo.H[l] + 3) / 4) * ((geo.W[l] + 7) / 8);
    const int64_t nb = T * d.M * d.N;
    if (nb > 0x7fffffff) return m2f::fail(M2F_EUNSUPPORTED, "%s: too many workgroups", fn);
    const unsigned tg = static_cast<unsigned>(nb);
#define M2F_FFT(LT)                                                                                           \
  (off32 ? msda_fused_fwd<LT, true, true><<<tg, 256, 0, st>>>(value, fe, geo, d.npairs(), d.S, d.M, d.Lq, output)  \
         : msda_fused_fwd<LT, true, false><<<tg, 256, 0, st>>>(value, fe, geo, d.npairs(), d.S, d.M, d.Lq, output))
    switch (d.L) {
      case 1: M2F_FFT(1); break;
      case 2: M2F_FFT(2); break;
      case 3: M2F_FFT(3); break;
      default: M2F_FFT(4); break;
    }
#undef M2F_FFT
    return m2f::check_launch(fn);
  }
  const unsigned grid = m2f::ceil_div(d.npairs(), 32);
#define M2F_FF(LT)                                                                                            \
  (off32 ? msda_fused_fwd<LT, false, true><<<grid, 256, 0, st>>>(value, fe, geo, d.npairs(), d.S, d.M, d.Lq, output) \
         : msda_fused_fwd<LT, false, false><<<grid, 256, 0, st>>>(value, fe, geo, d.npairs(), d.S, d.M, d.Lq, output))
  switch (d.L) {
    case 1: M2F_FF(1); break;
    case 2: M2F_FF(2); break;
    case 3: M2F_FF(3); break;
    default: M2F_FF(4); break;
  }
#undef M2F_FF
  return m2f::check_launch(fn);
}

extern "C" int m2f_msda_fused_bwd_workspace(const int64_t* host_spatial_shapes, int batch, int spatial_size,
                                            int num_heads, int channels, int num_levels, int num_point,
                                            int64_t* workspace_bytes) {
  const char* fn = "m2f_msda_fused_bwd_workspace";
  const Dims d{batch, spatial_size, num_heads, channels, num_levels, spatial_size, num_point};
  if (!host_spatial_shapes || !workspace_bytes) return m2f::fail(M2F_EINVAL, "%s: null pointer", fn);
  TileGeom geo;
  size_t lds;
  int threads;
  if (!make_tile_geom(d, host_spatial_shapes, geo, lds, threads))
    return m2f::fail(M2F_EUNSUPPORTED, "%s: needs the encoder layout", fn);
  // deterministic mode (msda_bwd_det): the int64 grad_value accumulator and two scale words; otherwise none
  *workspace_bytes = m2f::option(m2f::kOptMsdaBwdDet, 0) != 0 ? det_workspace_bytes(d) : 0;
  return m2f::ok();
}

static int fused_bwd(int hm, const char* fn, const float* value, const float* proj, int proj_ld, const float* ref,
                                      int64_t ref_batch_stride, const int64_t* host_spatial_shapes,
                                      const float* grad_output, int batch, int spatial_size, int num_heads,
                                      int channels, int num_levels, int num_query, int num_point,
                                      float* grad_value, float* grad_proj, void* workspace, int64_t workspace_bytes,
                                      void* stream) {
  const Dims d{batch, spatial_size, num_heads, channels, num_levels, num_query, num_point};
  TileGeom geo0;
  int rc = fused_check(fn, value, proj, proj_ld, ref, host_spatial_shapes, d, geo0);
  if (rc) return rc;
  if (!grad_output || !grad_value || !grad_proj || !m2f::aligned(grad_output, 16) || !m2f::aligned(grad_value, 16))
    return m2f::fail(M2F_EINVAL, "%s: bad gradient pointer", fn);
  TileGeom geo;
  size_t lds;
  int threads;
  if (!make_tile_geom(d, host_spatial_shapes, geo, lds, threads))
    return m2f::fail(M2F_EUNSUPPORTED, "%s: needs the encoder layout (num_query == spatial_size), value under 2 GiB "
                     "and levels under 2^24 pixels", fn);
  hipStream_t st = static_cast<hipStream_t>(stream);
  const int64_t nval = static_cast<int64_t>(d.N) * d.S * d.M * d.D;
  const size_t gv_bytes = static_cast<size_t>(nval) * sizeof(float);
  hipError_t e = m2f::zero_async(grad_value, gv_bytes, st);
  if (e != hipSuccess) return m2f::fail(M2F_ELAUNCH, "%s: memset grad_value: %s", fn, hipGetErrorString(e));
  const FrontEnd fe{proj, proj_ld, ref, ref_batch_stride, hm};
  DetBufs det;
  if (m2f::option(m2f::kOptMsdaBwdDet, 0) != 0) {
    const int64_t need = det_workspace_bytes(d);
    if (!workspace || workspace_bytes < need || !m2f::aligned(workspace, 16))
      return m2f::fail(M2F_EINVAL, "%s: deterministic mode needs a 16-byte aligned workspace of %lld bytes "
                       "(m2f_msda_fused_bwd_workspace)", fn, static_cast<long long>(need));
    det.acc = static_cast<unsigned long long*>(workspace);
    det.scale = reinterpret_cast<unsigned*>(det.acc + nval);
    e = m2f::zero_async(workspace, static_cast<size_t>(need), st);
    if (e != hipSuccess) return m2f::fail(M2F_ELAUNCH, "%s: memset workspace: %s", fn, hipGetErrorString(e));
    const int64_t n4 = static_cast<int64_t>(d.N) * d.Lq * d.M * d.D / 4;  // grad_output (N, Lq, M*32) fp32
    msda_det_scale_kernel<<<2048, 256, 0, st>>>(reinterpret_cast<const float4*>(grad_output), n4, det.scale);
  }
  if (int trc = launch_tiled_levels<true>(value, nullptr, nullptr, fe, grad_output, geo, lds, threads, d, grad_value,
                                          grad_proj, nullptr, st, det))
    return trc;
  if (det.acc)
    msda_det_convert_kernel<<<4096, 256, 0, st>>>(reinterpret_cast<const long long*>(det.acc), nval, d.Lq, det.scale,
                                                  grad_value);
  return m2f::check_launch(fn);
}

extern "C" int m2f_msda_fused_fwd_f32(const float* value, const float* proj, int proj_ld, const float* ref,
                                      int64_t ref_batch_stride, const int64_t* host_spatial_shapes, int batch,
                                      int spatial_size, int num_heads, int channels, int num_levels,
                                      int num_query, int num_point, float* output, void* stream) {
  return fused_fwd(0, "m2f_msda_fused_fwd_f32", value, proj, proj_ld, ref, ref_batch_stride, host_spatial_shapes,
                   batch, spatial_size, num_heads, channels, num_levels, num_query, num_point, output, stream);
}

extern "C" int m2f_msda_fused_fwd_hm_f32(const float* value, const float* proj, int proj_ld, const float* ref,
                                      int64_t ref_batch_stride, const int64_t* host_spatial_shapes, int batch,
                                      int spatial_size, int num_heads, int channels, int num_levels,
                                      int num_query, int num_point, float* output, void* stream) {
  return fused_fwd(1, "m2f_msda_fused_fwd_hm_f32", value, proj, proj_ld, ref, ref_batch_stride, host_spatial_shapes,
                   batch, spatial_size, num_heads, channels, num_levels, num_query, num_point, output, stream);
}

extern "C" int m2f_msda_fused_bwd_f32(const float* value, const float* proj, int proj_ld, const float* ref,
                                      int64_t ref_batch_stride, const int64_t* host_spatial_shapes,
                                      const float* grad_output, int batch, int spatial_size, int num_heads,
                                      int channels, int num_levels, int num_query, int num_point,
                                      float* grad_value, float* grad_proj, void* workspace, int64_t workspace_bytes,
                                      void* stream) {
  return fused_bwd(0, "m2f_msda_fused_bwd_f32", value, proj, proj_ld, ref, ref_batch_stride, host_spatial_shapes,
                   grad_output, batch, spatial_size, num_heads, channels, num_levels, num_query, num_point,
                   grad_value, grad_proj, workspace, workspace_bytes, stream);
}

extern "C" int m2f_msda_fused_bwd_hm_f32(const float* value, const float* proj, int proj_ld, const float* ref,
                                      int64_t ref_batch_stride, const int64_t* host_spatial_shapes,
                                      const float* grad_output, int batch, int spatial_size, int num_heads,
                                      int channels, int num_levels, int num_query, int num_point,
                                      float* grad_value, float* grad_proj, void* workspace, int64_t workspace_bytes,
                                      void* stream) {
  return fused_bwd(1, "m2f_msda_fused_bwd_hm_f32", value, proj, proj_ld, ref, ref_batch_stride, host_spatial_shapes,
                   grad_output, batch, spatial_size, num_heads, channels, num_levels, num_query, num_point,
                   grad_value, grad_proj, workspace, workspace_bytes, stream);
}

#ifdef M2F_DIAG
// Diagnostic build only (tools/msda_stamps.py builds it as a separate library): the unfused tiled backward with
// s_memtime stamps at its phase barriers, stamps[wg * 8 + k], k = 0..4.
extern "C" int m2f_diag_msda_bwd_stamps_f32(const float* value, const float* loc, const float* attn,
                                            const float* grad_output, int batch, int spatial_size, int num_heads,
                                            int num_levels, const int64_t* host_spatial_shapes, float* grad_value,
                                            float* grad_loc, float* grad_attn, unsigned long long* stamps,
                                            int noflush, void* stream) {
  const Dims d{batch, spatial_size, num_heads, 32, num_levels, spatial_size, 4};
  TileGeom geo;
  size_t lds;
  int threads;
  if (num_levels != 3 || !make_tile_geom(d, host_spatial_shapes, geo, lds, threads))
    return m2f::fail(M2F_EUNSUPPORTED, "diag");
  hipStream_t st = static_cast<hipStream_t>(stream);
  (void)m2f::zero_async(grad_value, static_cast<size_t>(d.N) * d.S * d.M * 32 * 4, st);
  const dim3 grid(geo.nty * geo.ntx * d.M * d.N);
#define M2F_DIAG_LAUNCH(TPB, NF)                                                                                  \
  do {                                                                                                           \
    (void)hipFuncSetAttribute(reinterpret_cast<const void*>(&msda_bwd_f32_tiled<3, false, TPB, false, false, true, NF>),      \
                              hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024 - 1024);                   \
    msda_bwd_f32_tiled<3, false, TPB, false, false, true, NF><<<grid, TPB, lds, st>>>(value, loc, attn, FrontEnd{}, grad_output, \
                                                                       geo, d.S, d.M, grad_value, grad_loc,     \
                                                                       grad_attn, nullptr, nullptr, stamps);    \
  } while (0)
  if (threads == 1024) {
    if (noflush) M2F_DIAG_LAUNCH(1024, true); else M2F_DIAG_LAUNCH(1024, false);
  } else {
    if (noflush) M2F_DIAG_LAUNCH(512, true); else M2F_DIAG_LAUNCH(512, false);
  }
#undef M2F_DIAG_LAUNCH
  return m2f::check_launch("m2f_diag_msda_bwd_stamps_f32");
}
#endif
