// fp32 convolutions of the pixel decoder's dense tail on the x3 (three-way split-bf16, fp32-accurate)
// MFMA engine, NCHW, stride 1, kernel 1x1 or 3x3 with "same" padding (msdeformattn.py:213-230 input_proj,
// :257-292 adapter_1 / layer_1, :245-252 mask_features; run in fp32 with autocast off, :314,320).
//
// Forward and input gradient are one implicit GEMM each, per image n:
//     O[co][p] = sum_{tap, ci} W[co][ci][tap] . I[ci][p + s(tap)]          (zero outside the image)
// i.e. C[p][co] = sum_k A[k][p] B[k][co] with k = (tap, ci): the pixel side is A (wave-direct: lane =
// pixel, 8 consecutive ci of one tap = 8 loads of 128-byte pixel rows across the wave), the weights are
// B (split once per call into the swizzled chunk images of the GEMM kernels, copied to LDS linearly).
// The input gradient is the same kernel on dO with the taps mirrored: s(T-1-t) = -s(t).
// Output tiles leave transposed through a per-wave LDS image: float4 runs along pixels of one channel.
//
// Weight gradient: dW[co][ci][tap] = sum_{n, p} dO[n][co][p] . I[n][ci][p + s(tap)], split over pixels
// (slabs reduced in a fixed order, deterministic): the (tap, ci) side is wave-direct (8 consecutive
// pixels of one shifted channel per lane), dO goes through LDS (a thread owns one channel x 8 pixels:
// two float4 loads), bias gradient = channel sums of dO taken while staging.
#include "bm2f.h"
#include "common.h"
#include "x3_device.h"

#include <hip/hip_runtime.h>

#include <type_traits>

namespace {

using namespace m2f_x3;

__device__ __forceinline__ void tap_shift(int T, int tap, int& dy, int& dx) {
  dy = T == 9 ? tap / 3 - 1 : 0;
  dx = T == 9 ? tap % 3 - 1 : 0;
}

// 16-bit activations (the backbone's autocast features, 1x1 convs only): the reference upcasts them with .float()
// (msdeformattn.py:320, 336), an exact conversion, so the kernels read them as they are and convert in registers;
// the input gradient goes back rounded to the feature dtype (round-to-nearest-even, as the cast's backward).
template <typename TI>
__device__ __forceinline__ float lo16(unsigned u) {
  if constexpr (std::is_same<TI, _Float16>::value)
    return static_cast<float>(__builtin_bit_cast(_Float16, static_cast<unsigned short>(u & 0xffffu)));
  else
    return __uint_as_float(u << 16);
}
template <typename TI>
__device__ __forceinline__ float hi16(unsigned u) {
  if constexpr (std::is_same<TI, _Float16>::value)
    return static_cast<float>(__builtin_bit_cast(_Float16, static_cast<unsigned short>(u >> 16)));
  else
    return __uint_as_float(u & 0xffff0000u);
}
template <typename TI>
__device__ __forceinline__ float to_f(TI v) {
  if constexpr (std::is_same<TI, float>::value) return v;
  else return static_cast<float>(v);
}
// two floats -> one word of two 16-bit values (element 0 in the low half)
template <typename TO>
__device__ __forceinline__ unsigned pack2(float a, float b) {
  using h2 = TO __attribute__((ext_vector_type(2)));
  return __builtin_bit_cast(unsigned, h2{static_cast<TO>(a), static_cast<TO>(b)});
}

// a lane's 8 A values in flight (loaded in one pipeline step, converted in the next): fp32 or 16-bit scalars
// (channel-strided NCHW reads), or one 16-byte vector of 8 consecutive channels (NHWC, 16-bit)
template <typename TI, bool NHWC>
struct ARaw {
  TI v[8];
  __device__ __forceinline__ void load(const TI* src, int64_t stride) {
#pragma unroll
    for (int e = 0; e < 8; ++e) v[e] = src[static_cast<int64_t>(e) * stride];
  }
  __device__ __forceinline__ void get(float (&x)[8]) const {
#pragma unroll
    for (int e = 0; e < 8; ++e) x[e] = to_f(v[e]);
  }
};
template <typename TI>
struct ARaw<TI, true> {
  using u4 = unsigned __attribute__((ext_vector_type(4)));
  u4 v;
  __device__ __forceinline__ void load(const TI* src, int64_t) { v = *reinterpret_cast<const u4*>(src); }
  __device__ __forceinline__ void get(float (&x)[8]) const {
#pragma unroll
    for (int p = 0; p < 4; ++p) {
      x[2 * p] = lo16<TI>(v[p]);
      x[2 * p + 1] = hi16<TI>(v[p]);
    }
  }
};

// Bs[c][p][n][16] (swizzled rows, NP rows) for the conv GEMM.  Chunk c holds channels 16 (c / T) .. +15 of
// tap c % T: the taps of one channel group are adjacent in k, so the pixel rows a block loads for one tap are
// re-read by the next taps from L1/L2 (tap-major k swept all channels per tap: the 3x3 forward then fetched
// its input about ten times from HBM, r02_a).
// mode 0 (forward):  n = co, Ca = Ci, value W[co][ci][tap]
// mode 1 (dgrad):    n = ci, Ca = Co, value W[co][ci][T-1-tap]
__global__ void __launch_bounds__(256) x3_conv_presplit(const float* __restrict__ Wt, int Co, int Ci, int T, int mode,
                                                        int NP, int nchunks, __bf16* __restrict__ Bs) {
  const int64_t t = blockIdx.x * static_cast<int64_t>(blockDim.x) + threadIdx.x;
  if (t >= static_cast<int64_t>(nchunks) * NP) return;
  const int c = static_cast<int>(t / NP), n = static_cast<int>(t - static_cast<int64_t>(c) * NP);
  const int Ca = mode == 0 ? Ci : Co, Nn = mode == 0 ? Co : Ci;
  bf8 pl[3][2];
#pragma unroll
  for (int j = 0; j < 16; ++j) {
    const int tap = c % T, ca = (c / T) * 16 + j;
    float v = 0.f;
    if (n < Nn && tap < T) {
      const int co = mode == 0 ? n : ca, ci = mode == 0 ? ca : n, tp = mode == 0 ? tap : T - 1 - tap;
      v = Wt[(static_cast<int64_t>(co) * Ci + ci) * T + tp];
    }
    __bf16 h, m, l;
    split3(v, h, m, l);
    pl[0][j >> 3][j & 7] = h;
    pl[1][j >> 3][j & 7] = m;
    pl[2][j >> 3][j & 7] = l;
  }
  const int sw = swz(n);
#pragma unroll
  for (int p = 0; p < 3; ++p) {
    bf8* dst = reinterpret_cast<bf8*>(Bs + ((static_cast<int64_t>(c) * 3 + p) * NP + n) * 16);
    dst[sw] = pl[p][0];
    dst[sw ^ 1] = pl[p][1];
  }
}

// ---------------------------------------------------------------------------------------------------
// forward / input gradient.  grid (HW / 128, ceil(Cout / 256), N); 4 waves x 32 pixels; Cout tile 256.
// ---------------------------------------------------------------------------------------------------
// TI / INHWC: the A operand's type and layout (16-bit and NHWC: T == 1 forward only); TO / ONHWC: the output's
// (16-bit and NHWC: T == 1 input gradient only)
template <int T, typename TI = float, typename TO = float, bool INHWC = false, bool ONHWC = false>
__global__ void __launch_bounds__(256, 2) x3_conv_kernel(const TI* __restrict__ I, int Ca, int H, int W,
                                                         const __bf16* __restrict__ Bs, int NP,
                                                         const float* __restrict__ bias, TO* __restrict__ O,
                                                         int Cout) {
  static_assert(T == 1 || (std::is_same<TI, float>::value && std::is_same<TO, float>::value && !INHWC && !ONHWC),
                "16-bit / NHWC operands: 1x1 only");
  static_assert(!(INHWC && std::is_same<TI, float>::value) && !(ONHWC && std::is_same<TO, float>::value),
                "NHWC operands are 16-bit");
  constexpr int NW = 4, NT = 256, BN = 256, TJ = BN / 32;
  constexpr int PIECES = 3 * BN * 2, NBL = PIECES / NT;
  constexpr int CHUNK = 3 * BN * 16;
  constexpr int EP = 36;
  constexpr int LDS_B = 2 * CHUNK * 2, LDS_E = NW * 32 * EP * 4;
  __shared__ __attribute__((aligned(16))) char smem[LDS_B > LDS_E ? LDS_B : LDS_E];
  __bf16(*sb)[CHUNK] = reinterpret_cast<__bf16(*)[CHUNK]>(smem);

  const int HW = H * W;
  // 3x3: 1-D grid with the grouped XCD remap (runs of 16 pixel tiles = 8 rows at W = 256 per XCD), so the
  // rows a tap shares with the neighbouring tiles are fetched into one L2 instead of three (fetch 4.5 -> 1.6 GB
  // per launch at config 2).  1x1 has no such reuse and keeps the 3-D grid (its 252 VGPRs leave no room for
  // the index math: it spilled and ran 2.9x slower)
  int n, n20, p0;
  if constexpr (T == 9) {
    const int np = HW / 128, nct = (Cout + BN - 1) / BN;
    const int id = xcd_group_remap(blockIdx.x, gridDim.x, 16);
    const int pt = id % np, rest = id / np;
    n = rest / nct;
    n20 = (rest - n * nct) * BN;
    p0 = pt * 128;
  } else {
    n = blockIdx.z;
    n20 = blockIdx.y * BN;
    p0 = blockIdx.x * 128;
  }
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const int li = lane & 31, lh = lane >> 5;
  const int pix = p0 + w * 32 + li, py = pix / W, px = pix - py * W;
  const TI* In = I + static_cast<int64_t>(n) * Ca * HW;
  const int cpt = Ca / kBK;               // chunks per tap
  const int nk = T * cpt;

  struct Regs {
    ARaw<TI, INHWC> a;
    bf8 b[NBL];
  };
  auto gload = [&](Regs& r, int c) {
    const int cc = min(c, nk - 1);
    // channel-group major for 3x3; 1x1 keeps the old form (its allocation sits at 252 VGPRs: the compiler
    // spilled 53 on the equivalent cc * 16)
    const int tap = T == 9 ? cc % T : cc / cpt;
    const int ci0 = (T == 9 ? cc / T : cc - tap * cpt) * kBK + lh * 8;
    int dy, dx;
    tap_shift(T, tap, dy, dx);
    const int yy = py + dy, xx = px + dx;
    const bool ok = yy >= 0 && yy < H && xx >= 0 && xx < W;
    if constexpr (INHWC) {
      r.a.load(In + static_cast<int64_t>(pix) * Ca + ci0, 1);
    } else {
      r.a.load(In + static_cast<int64_t>(ci0) * HW + (ok ? yy * W + xx : 0), HW);
    }
    const __bf16* bc = Bs + static_cast<int64_t>(cc) * 3 * NP * 16;
#pragma unroll
    for (int u = 0; u < NBL; ++u) {
      const int q = tid + u * NT, p = q / (BN * 2), rem = q - p * BN * 2;
      r.b[u] = *reinterpret_cast<const bf8*>(bc + (static_cast<int64_t>(p) * NP + n20) * 16 + rem * 8);
    }
  };
  auto bstore = [&](const Regs& r, int buf) {
#pragma unroll
    for (int u = 0; u < NBL; ++u) *reinterpret_cast<bf8*>(&sb[buf][(tid + u * NT) * 8]) = r.b[u];
  };
  auto asplit = [&](const Regs& r, int c, bf8 (&fa)[3]) {
    const int tap = T == 9 ? c % T : c / cpt;
    int dy, dx;
    tap_shift(T, tap, dy, dx);
    const int yy = py + dy, xx = px + dx;
    const bool ok = yy >= 0 && yy < H && xx >= 0 && xx < W;
    float v[8];
    r.a.get(v);
#pragma unroll
    for (int e = 0; e < 8; ++e) v[e] = ok ? v[e] : 0.f;
    split8(v, fa);
  };

  f16v acc[TJ];
#pragma unroll
  for (int j = 0; j < TJ; ++j)
#pragma unroll
    for (int e = 0; e < 16; ++e) acc[j][e] = 0.f;
  const int boff = li * 16 + ((lh ^ swz(li)) * 8);
  auto chunk_mfma = [&](int buf, const bf8 (&fa)[3]) {
    const __bf16* base = &sb[buf][0];
#pragma unroll
    for (int j = 0; j < TJ; ++j) {
      const int off = j * 32 * 16 + boff;
      acc[j] = mfma_x3(fa, *reinterpret_cast<const bf8*>(base + off), *reinterpret_cast<const bf8*>(base + BN * 16 + off),
                       *reinterpret_cast<const bf8*>(base + 2 * BN * 16 + off), acc[j]);
    }
  };

  Regs r0, r1;
  bf8 fa[3];
  gload(r0, 0);
  gload(r1, 1);
  bstore(r0, 0);
  asplit(r0, 0, fa);
  __syncthreads();
  // (a two-fragment-set branch-free pipeline with the split kept before the barrier, which gains 3-7 % in
  // x3_tn_kernel, measured +1.7 % here: r2ao)
  {
    auto step = [&](int c, Regs& cur, Regs& nxt) {
      if (c + 2 < nk) gload(cur, c + 2);
      M2F_X3_PREFETCH_FENCE();
      chunk_mfma(c & 1, fa);
      if (c + 1 < nk) {
        bstore(nxt, (c + 1) & 1);
        asplit(nxt, c + 1, fa);
      }
      __syncthreads();
    };
    for (int c = 0; c < nk; c += 2) {
      step(c, r0, r1);
      if (c + 1 < nk) step(c + 1, r1, r0);
    }
  }

  // epilogue: tile j holds C[pixel = (e&3)+8(e>>2)+4lh][co = li]; the image is stored transposed
  // ([co][pixel]) and read back as float4 runs of pixels
  float* img = reinterpret_cast<float*>(smem) + w * 32 * EP;
  TO* Ob = O + static_cast<int64_t>(n) * Cout * HW;
  const int er = lane >> 3, ec = (lane & 7) * 4;
#pragma unroll
  for (int j = 0; j < TJ; ++j) {
    if constexpr (ONHWC) {
      // pixel-major image [pixel][co] (row stride 33), read back as 8 consecutive channels of one pixel: a 16-byte
      // store of 8 16-bit values, 4 lanes per pixel row of the tile
#pragma unroll
      for (int e = 0; e < 16; ++e) img[((e & 3) + 8 * (e >> 2) + 4 * lh) * 33 + li] = acc[j][e];
    } else {
#pragma unroll
      for (int e = 0; e < 16; ++e) img[li * EP + (e & 3) + 8 * (e >> 2) + 4 * lh] = acc[j][e];
    }
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    if constexpr (ONHWC) {
      using u4 = unsigned __attribute__((ext_vector_type(4)));
#pragma unroll
      for (int it = 0; it < 2; ++it) {
        const int item = lane + 64 * it, pr = item >> 2, grp = item & 3, co = n20 + j * 32 + grp * 8;
        const float* s = &img[pr * 33 + grp * 8];
        if (co < Cout) {
          const u4 pk = {pack2<TO>(s[0], s[1]), pack2<TO>(s[2], s[3]), pack2<TO>(s[4], s[5]), pack2<TO>(s[6], s[7])};
          *reinterpret_cast<u4*>(O + (static_cast<int64_t>(n) * HW + p0 + w * 32 + pr) * Cout + co) = pk;
        }
      }
    } else {
      // the 4 output channels' biases loaded before any is used (behind the range test, each load had been a
      // memory round trip of its own)
      float bq[4] = {0.f, 0.f, 0.f, 0.f};
      if (bias) {
#pragma unroll
        for (int q = 0; q < 4; ++q) bq[q] = bias[min(n20 + j * 32 + q * 8 + er, Cout - 1)];
      }
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const int lr = q * 8 + er, co = n20 + j * 32 + lr;
        f4 v = *reinterpret_cast<const f4*>(&img[lr * EP + ec]);
        if (co < Cout) {
          if (bias) v += bq[q];
          TO* dst = Ob + static_cast<int64_t>(co) * HW + p0 + w * 32 + ec;
          if constexpr (std::is_same<TO, float>::value) {
            *reinterpret_cast<f4*>(dst) = v;
          } else {
            using u2 = unsigned __attribute__((ext_vector_type(2)));
            *reinterpret_cast<u2*>(dst) = u2{pack2<TO>(v[0], v[1]), pack2<TO>(v[2], v[3])};
          }
        }
      }
    }
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
  }
}

// ---------------------------------------------------------------------------------------------------
// weight gradient.  C[(tap, ci)][co] over pixels m = (n, p), split into slabs of rows_per_split pixels
// (multiples of 16: a chunk never crosses an image).  Block: 4 waves x 32 (tap, ci) columns, 256 co.
// grid = splits * tiles, tiles = ceil(T*Ci / 128) * ceil(Co / 256).
// ---------------------------------------------------------------------------------------------------
// TI / INHWC: the input's type and layout (16-bit and NHWC: T == 1 only)
template <int T, typename TI = float, bool INHWC = false>
__global__ void __launch_bounds__(256, 2) x3_conv_wgrad_kernel(const float* __restrict__ dO,
                                                               const TI* __restrict__ I, int N, int Co, int Ci,
                                                               int H, int W, int rows_per_split,
                                                               float* __restrict__ slab, float* __restrict__ bias_slab) {
  constexpr int NW = 4, NT = 256, BN = 256, TJ = BN / 32;
  constexpr int JOBS = BN * 2, NJ = JOBS / NT;
  constexpr int CHUNK = 3 * BN * 16;
  constexpr int EP = 36;
  constexpr int LDS_B = 2 * CHUNK * 2, LDS_E = NW * 32 * EP * 4;
  __shared__ __attribute__((aligned(16))) char smem[LDS_B > LDS_E ? LDS_B : LDS_E];
  __bf16(*sb)[CHUNK] = reinterpret_cast<__bf16(*)[CHUNK]>(smem);

  const int HW = H * W;
  const int64_t M = static_cast<int64_t>(N) * HW;
  const int N1 = T * Ci;
  const int nb1 = (N1 + 127) / 128, nb2 = (Co + BN - 1) / BN, tiles = nb1 * nb2;
  const int id = xcd_remap(blockIdx.x, gridDim.x);
  const int split = id / tiles, t = id % tiles;
  const int b1 = t / nb2, b2 = t % nb2;
  const int n10 = b1 * 128, n20 = b2 * BN;
  const int64_t r0 = static_cast<int64_t>(split) * rows_per_split;
  const int64_t r1 = min(M, r0 + rows_per_split);
  const int nk = r1 > r0 ? static_cast<int>((r1 - r0 + kBK - 1) / kBK) : 0;
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const int li = lane & 31, lh = lane >> 5;
  const int col = min(n10 + w * 32 + li, N1 - 1), tap = col / Ci, ci = col - tap * Ci;
  int dy, dx;
  tap_shift(T, tap, dy, dx);
  const bool csum = bias_slab != nullptr && b1 == 0;

  static_assert(T == 1 || (std::is_same<TI, float>::value && !INHWC), "16-bit / NHWC input: 1x1 only");
  constexpr bool k32 = std::is_same<TI, float>::value;
  struct Regs {
    f4 a[k32 ? 3 : 1];                      // fp32: 8 (1x1) or 12 (3x3) pixels of the lane's channel
    ARaw<TI, !INHWC> h;                     // 16-bit NCHW: one 16-byte vector of 8 pixels; NHWC: 8 strided scalars
    f4 b[NJ][2];
  };
  // chunk c: pixels m = r0 + 16c .. +15 of one image; lane rows 8lh .. 8lh+7 (same image row: W % 8 == 0).
  // A lane's 8 shifted pixels x0+dx .. x0+dx+7 come from three aligned float4 loads of its row (x0-4 ..
  // x0+7 for dx = -1, x0 .. x0+11 for dx = +1; two for dx = 0) instead of eight scalar loads: a quarter
  // of the address-unit work; the row edges are zeroed when the window is assembled (awin).
  auto gload = [&](Regs& r, int c) {
    const int64_t m = min(r0 + static_cast<int64_t>(c) * kBK, M - kBK);
    const int n = static_cast<int>(m / HW), p = static_cast<int>(m - static_cast<int64_t>(n) * HW);
    const int pa = p + lh * 8, y = pa / W, x0 = pa - y * W;
    const int yy = y + dy;
    if constexpr (!k32) {
      if constexpr (INHWC) r.h.load(I + (static_cast<int64_t>(n) * HW + pa) * Ci + ci, Ci);
      else r.h.load(I + (static_cast<int64_t>(n) * Ci + ci) * HW + pa, 1);
    } else if (T == 1) {
      const TI* row = I + (static_cast<int64_t>(n) * Ci + ci) * HW + static_cast<int64_t>(y) * W;
      r.a[0] = *reinterpret_cast<const f4*>(row + x0);
      r.a[1] = *reinterpret_cast<const f4*>(row + x0 + 4);
    } else {  // one code path for every tap: 12 pixels from base (x0 - 4, or x0 when dx = +1)
      const TI* row = I + (static_cast<int64_t>(n) * Ci + ci) * HW + static_cast<int64_t>(yy >= 0 && yy < H ? yy : y) * W;
      const int base = dx > 0 ? x0 : x0 - 4;
      r.a[0] = *reinterpret_cast<const f4*>(row + max(base, 0));
      r.a[1] = *reinterpret_cast<const f4*>(row + base + 4);
      r.a[2] = *reinterpret_cast<const f4*>(row + min(base + 8, W - 4));
    }
#pragma unroll
    for (int u = 0; u < NJ; ++u) {
      const int job = tid + u * NT, half = job / BN, co = min(n20 + job % BN, Co - 1);
      const float* gsrc = dO + (static_cast<int64_t>(n) * Co + co) * HW + p + half * 8;
      r.b[u][0] = *reinterpret_cast<const f4*>(gsrc);
      r.b[u][1] = *reinterpret_cast<const f4*>(gsrc + 4);
    }
  };
  float csb[NJ];
#pragma unroll
  for (int u = 0; u < NJ; ++u) csb[u] = 0.f;
  auto bstore = [&](const Regs& r, int c, int buf) {
    const bool live = r0 + static_cast<int64_t>(c) * kBK < r1;  // a clamped duplicate chunk contributes 0
#pragma unroll
    for (int u = 0; u < NJ; ++u) {
      const int job = tid + u * NT, half = job / BN, cl = job % BN;
      float v[8];
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        v[e] = live ? r.b[u][e >> 2][e & 3] : 0.f;
        if (csum) csb[u] += v[e];
      }
      bf8 pl[3];
      split8(v, pl);
      const int off = cl * 16 + ((half ^ swz(cl)) * 8);
      *reinterpret_cast<bf8*>(&sb[buf][off]) = pl[0];
      *reinterpret_cast<bf8*>(&sb[buf][BN * 16 + off]) = pl[1];
      *reinterpret_cast<bf8*>(&sb[buf][2 * BN * 16 + off]) = pl[2];
    }
  };
  auto asplit = [&](const Regs& r, int c, bf8 (&fa)[3]) {
    const int64_t m = r0 + static_cast<int64_t>(c) * kBK;
    const bool live = m < r1;
    const int64_t mc = min(m, M - kBK);
    const int n = static_cast<int>(mc / HW), p = static_cast<int>(mc - static_cast<int64_t>(n) * HW);
    const int pa = p + lh * 8, y = pa / W, x0 = pa - y * W, yy = y + dy;
    const bool rok = live && yy >= 0 && yy < H;
    float v[8];
    if constexpr (!k32) {
      r.h.get(v);
    } else if (T == 1) {
#pragma unroll
      for (int e = 0; e < 8; ++e) v[e] = r.a[e >> 2][e & 3];
    } else {
      // window start in the 12 loaded pixels: 3 (dx = -1), 4 (dx = 0), 1 (dx = +1); selects, no branches
      const int st = dx > 0 ? 1 : 4 + dx;
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        const float c1 = r.a[(e + 1) >> 2][(e + 1) & 3], c3 = r.a[(e + 3) >> 2][(e + 3) & 3];
        const float c4 = r.a[(e + 4) >> 2][(e + 4) & 3];
        v[e] = st == 1 ? c1 : (st == 3 ? c3 : c4);
      }
      if (dx < 0 && x0 == 0) v[0] = 0.f;      // left of the row
      if (dx > 0 && x0 + 8 >= W) v[7] = 0.f;  // right of the row
    }
#pragma unroll
    for (int e = 0; e < 8; ++e) v[e] = rok ? v[e] : 0.f;
    split8(v, fa);
  };

  f16v acc[TJ];
#pragma unroll
  for (int j = 0; j < TJ; ++j)
#pragma unroll
    for (int e = 0; e < 16; ++e) acc[j][e] = 0.f;
  const int boff = li * 16 + ((lh ^ swz(li)) * 8);
  auto chunk_mfma = [&](int buf, const bf8 (&fa)[3]) {
    const __bf16* base = &sb[buf][0];
#pragma unroll
    for (int j = 0; j < TJ; ++j) {
      const int off = j * 32 * 16 + boff;
      acc[j] = mfma_x3(fa, *reinterpret_cast<const bf8*>(base + off), *reinterpret_cast<const bf8*>(base + BN * 16 + off),
                       *reinterpret_cast<const bf8*>(base + 2 * BN * 16 + off), acc[j]);
    }
  };

  if (nk > 0) {
    Regs ra, rb;
    bf8 fa[3];
    gload(ra, 0);
    if (nk > 1) gload(rb, 1);
    bstore(ra, 0, 0);
    asplit(ra, 0, fa);
    __syncthreads();
    auto step = [&](int c, Regs& cur, Regs& nxt) {
      if (c + 2 < nk) gload(cur, c + 2);
      M2F_X3_PREFETCH_FENCE();
      chunk_mfma(c & 1, fa);
      if (c + 1 < nk) {
        bstore(nxt, c + 1, (c + 1) & 1);
        asplit(nxt, c + 1, fa);
      }
      __syncthreads();
    };
    for (int c = 0; c < nk; c += 2) {
      step(c, ra, rb);
      if (c + 1 < nk) step(c + 1, rb, ra);
    }
  }

  // slab[split][(tap, ci)][co]
  float* out = slab + static_cast<int64_t>(split) * N1 * Co;
  float* img = reinterpret_cast<float*>(smem) + w * 32 * EP;
  const int er = lane >> 3, ec = (lane & 7) * 4;
#pragma unroll
  for (int j = 0; j < TJ; ++j) {
#pragma unroll
    for (int e = 0; e < 16; ++e) img[((e & 3) + 8 * (e >> 2) + 4 * lh) * EP + li] = acc[j][e];
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const int lr = q * 8 + er, row = n10 + w * 32 + lr, cc = n20 + j * 32 + ec;
      const f4 v = *reinterpret_cast<const f4*>(&img[lr * EP + ec]);
      if (row < N1 && cc < Co) *reinterpret_cast<f4*>(out + static_cast<int64_t>(row) * Co + cc) = v;
    }
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
  }
  if (csum) {
    __syncthreads();
    float* red = reinterpret_cast<float*>(smem);
#pragma unroll
    for (int u = 0; u < NJ; ++u) {
      const int job = tid + u * NT;
      if (job / BN == 1) red[job % BN] = csb[u];
    }
    __syncthreads();
#pragma unroll
    for (int u = 0; u < NJ; ++u) {
      const int job = tid + u * NT, cc = n20 + job % BN;
      if (job / BN == 0 && cc < Co) bias_slab[static_cast<int64_t>(split) * Co + cc] = csb[u] + red[job % BN];
    }
  }
}

// out[r][c] = sum_s slab[s][r * ncols + c] (fixed order)
__global__ void __launch_bounds__(256) x3_conv_slab_reduce(const float* __restrict__ slab, int splits, int64_t n,
                                                           float* __restrict__ out) {
  const int64_t i = blockIdx.x * static_cast<int64_t>(blockDim.x) + threadIdx.x;
  if (i >= n) return;
  float a0 = 0.f, a1 = 0.f, a2 = 0.f, a3 = 0.f;
  int s = 0;
  for (; s + 3 < splits; s += 4) {
    a0 += slab[(s + 0) * n + i];
    a1 += slab[(s + 1) * n + i];
    a2 += slab[(s + 2) * n + i];
    a3 += slab[(s + 3) * n + i];
  }
  for (; s < splits; ++s) a0 += slab[s * n + i];
  out[i] = (a0 + a1) + (a2 + a3);
}

int conv_check(const char* fn, int N, int C, int H, int W, int Co, int T) {
  if (N <= 0 || C <= 0 || H <= 0 || W <= 0 || Co <= 0) return m2f::fail(M2F_EINVAL, "%s: bad sizes", fn);
  if (T != 1 && T != 9) return m2f::fail(M2F_EUNSUPPORTED, "%s: kernel must be 1x1 or 3x3", fn);
  if (C % 16 || (H * W) % 128 || W % 8)
    return m2f::fail(M2F_EUNSUPPORTED, "%s: needs channels %% 16 == 0, H*W %% 128 == 0, W %% 8 == 0", fn);
  return M2F_OK;
}

int64_t conv_ws(int Ca, int Nn, int T) {
  const int64_t NP = (Nn + 255) / 256 * 256, nchunks = static_cast<int64_t>(T) * Ca / kBK;
  return nchunks * 3 * NP * 16 * 2;
}

struct WgPlan {
  int splits, rows;
};

WgPlan wg_plan(int64_t M, int N1, int Co) {
  const int tiles = ((N1 + 127) / 128) * ((Co + 255) / 256);
  int64_t splits = (512 + tiles - 1) / tiles;
  const int64_t max_splits = (M + 8 * kBK - 1) / (8 * kBK);
  if (splits > max_splits) splits = max_splits;
  if (splits < 1) splits = 1;
  const int64_t r = (M + splits - 1) / splits;
  return WgPlan{static_cast<int>(splits), static_cast<int>((r + kBK - 1) / kBK * kBK)};
}

}  // namespace

extern "C" int m2f_conv_f32x3_workspace(int N, int Ci, int Co, int H, int W, int ksize, int64_t* workspace_bytes) {
  const int T = ksize * ksize;
  int rc = conv_check("m2f_conv_f32x3_workspace", N, Ci, H, W, Co, T);
  if (rc) return rc;
  if (Co % 16) return m2f::fail(M2F_EUNSUPPORTED, "m2f_conv_f32x3_workspace: out channels %% 16 != 0");
  const int64_t fwd = conv_ws(Ci, Co, T), dgrad = conv_ws(Co, Ci, T);
  const WgPlan p = wg_plan(static_cast<int64_t>(N) * H * W, T * Ci, Co);
  const int64_t wgrad = static_cast<int64_t>(p.splits) * (static_cast<int64_t>(T) * Ci * Co + Co) * 4;
  int64_t m = fwd > dgrad ? fwd : dgrad;
  if (wgrad > m) m = wgrad;
  if (workspace_bytes) *workspace_bytes = m;
  return m2f::ok();
}

namespace {

// 1x1 launches with 16-bit / NHWC operands (mode 0: the input; mode 1: the output)
template <typename TI, typename TO, bool INHWC, bool ONHWC>
void launch_1x1(const void* I, int Ca, int H, int W, const __bf16* Bs, int NP, const float* bias, void* O, int Nn, int N,
                hipStream_t st) {
  const dim3 grid((H * W) / 128, (Nn + 255) / 256, N);
  x3_conv_kernel<1, TI, TO, INHWC, ONHWC><<<grid, 256, 0, st>>>(static_cast<const TI*>(I), Ca, H, W, Bs, NP, bias,
                                                                 static_cast<TO*>(O), Nn);
}

int conv_impl(const char* fn, const void* I, int i_dtype, int i_nhwc, const float* Wt, const float* bias, void* O,
              int o_dtype, int o_nhwc, int N, int Ci, int Co, int H, int W, int ksize, int mode, void* workspace,
              int64_t workspace_bytes, void* stream) {
  const int T = ksize * ksize;
  int rc = conv_check(fn, N, mode == 0 ? Ci : Co, H, W, mode == 0 ? Co : Ci, T);
  if (rc) return rc;
  if (!I || !Wt || !O || !workspace) return m2f::fail(M2F_EINVAL, "%s: null pointer", fn);
  if (mode != 0 && mode != 1) return m2f::fail(M2F_EINVAL, "%s: mode %d", fn, mode);
  if (mode == 1 && bias) return m2f::fail(M2F_EINVAL, "%s: the input gradient takes no bias", fn);
  const bool i16 = i_dtype == M2F_F16 || i_dtype == M2F_BF16, o16 = o_dtype == M2F_F16 || o_dtype == M2F_BF16;
  if ((i_dtype != M2F_F32 && !i16) || (o_dtype != M2F_F32 && !o16)) return m2f::fail(M2F_EINVAL, "%s: dtype", fn);
  // the forward reads 16-bit / NHWC activations and writes fp32 NCHW; the input gradient reads fp32 NCHW and
  // writes 16-bit / NHWC; both only for 1x1, NHWC only for 16-bit
  const bool io_ok = mode == 0 ? (o_dtype == M2F_F32 && !o_nhwc && (!i_nhwc || i16))
                               : (i_dtype == M2F_F32 && !i_nhwc && (!o_nhwc || o16));
  if (!io_ok || ((i16 || o16 || i_nhwc || o_nhwc) && T != 1))
    return m2f::fail(M2F_EUNSUPPORTED, "%s: operand types / layouts (in %d/%d, out %d/%d, %dx%d, mode %d)", fn, i_dtype,
                     i_nhwc, o_dtype, o_nhwc, ksize, ksize, mode);
  if (!m2f::aligned(O, 16) || !m2f::aligned(workspace, 16) || (i_nhwc && !m2f::aligned(I, 16)))
    return m2f::fail(M2F_EINVAL, "%s: misaligned", fn);
  const int Ca = mode == 0 ? Ci : Co, Nn = mode == 0 ? Co : Ci;
  // the 16-bit / NHWC epilogues store 8 output channels per 16-byte write, guarded per group start only: the
  // output channel count must be whole 16-channel groups (conv_check validates the A operand's channels only)
  if ((i16 || o16 || i_nhwc || o_nhwc) && Nn % 16)
    return m2f::fail(M2F_EUNSUPPORTED, "%s: 16-bit / NHWC operands need output channels %% 16 == 0 (got %d)", fn, Nn);
  if (workspace_bytes < conv_ws(Ca, Nn, T)) return m2f::fail(M2F_EINVAL, "%s: workspace too small", fn);
  hipStream_t st = static_cast<hipStream_t>(stream);
  const int NP = (Nn + 255) / 256 * 256, nchunks = T * Ca / kBK;
  __bf16* Bs = static_cast<__bf16*>(workspace);
  x3_conv_presplit<<<m2f::ceil_div(static_cast<int64_t>(nchunks) * NP, 256), 256, 0, st>>>(Wt, Co, Ci, T, mode, NP,
                                                                                          nchunks, Bs);
  if ((rc = m2f::check_launch(fn))) return rc;
  if (T == 9) {
    const int64_t nblk = static_cast<int64_t>((H * W) / 128) * ((Nn + 255) / 256) * N;
    if (nblk > 0x7fffffff) return m2f::fail(M2F_EUNSUPPORTED, "%s: too many tiles", fn);
    x3_conv_kernel<9><<<static_cast<unsigned>(nblk), 256, 0, st>>>(static_cast<const float*>(I), Ca, H, W, Bs, NP,
                                                                    bias, static_cast<float*>(O), Nn);
  } else if (mode == 0) {
    if (i_dtype == M2F_F32) launch_1x1<float, float, false, false>(I, Ca, H, W, Bs, NP, bias, O, Nn, N, st);
    else if (i_dtype == M2F_F16 && i_nhwc) launch_1x1<_Float16, float, true, false>(I, Ca, H, W, Bs, NP, bias, O, Nn, N, st);
    else if (i_dtype == M2F_F16) launch_1x1<_Float16, float, false, false>(I, Ca, H, W, Bs, NP, bias, O, Nn, N, st);
    else if (i_nhwc) launch_1x1<__bf16, float, true, false>(I, Ca, H, W, Bs, NP, bias, O, Nn, N, st);
    else launch_1x1<__bf16, float, false, false>(I, Ca, H, W, Bs, NP, bias, O, Nn, N, st);
  } else {
    if (o_dtype == M2F_F32) launch_1x1<float, float, false, false>(I, Ca, H, W, Bs, NP, bias, O, Nn, N, st);
    else if (o_dtype == M2F_F16 && o_nhwc) launch_1x1<float, _Float16, false, true>(I, Ca, H, W, Bs, NP, bias, O, Nn, N, st);
    else if (o_dtype == M2F_F16) launch_1x1<float, _Float16, false, false>(I, Ca, H, W, Bs, NP, bias, O, Nn, N, st);
    else if (o_nhwc) launch_1x1<float, __bf16, false, true>(I, Ca, H, W, Bs, NP, bias, O, Nn, N, st);
    else launch_1x1<float, __bf16, false, false>(I, Ca, H, W, Bs, NP, bias, O, Nn, N, st);
  }
  return m2f::check_launch(fn);
}

template <typename TI, bool INHWC>
void launch_wgrad(int T, unsigned grid, const float* dO, const void* I, int N, int Co, int Ci, int H, int W, int rows,
                  float* slab, float* bslab, hipStream_t st) {
  if (T == 9)
    x3_conv_wgrad_kernel<9><<<grid, 256, 0, st>>>(dO, static_cast<const float*>(I), N, Co, Ci, H, W, rows, slab, bslab);
  else
    x3_conv_wgrad_kernel<1, TI, INHWC><<<grid, 256, 0, st>>>(dO, static_cast<const TI*>(I), N, Co, Ci, H, W, rows, slab,
                                                             bslab);
}

int wgrad_impl(const char* fn, const float* dO, const void* I, int i_dtype, int i_nhwc, float* dW, float* dbias, int N,
               int Ci, int Co, int H, int W, int ksize, void* workspace, int64_t workspace_bytes, void* stream) {
  const int T = ksize * ksize;
  int rc = conv_check(fn, N, Ci, H, W, Co, T);
  if (rc) return rc;
  if (Co % 16) return m2f::fail(M2F_EUNSUPPORTED, "%s: out channels %% 16 != 0", fn);
  if (!dO || !I || !dW || !workspace) return m2f::fail(M2F_EINVAL, "%s: null pointer", fn);
  const bool i16 = i_dtype == M2F_F16 || i_dtype == M2F_BF16;
  if (i_dtype != M2F_F32 && !i16) return m2f::fail(M2F_EINVAL, "%s: dtype", fn);
  if ((i16 || i_nhwc) && (T != 1 || !i16))
    return m2f::fail(M2F_EUNSUPPORTED, "%s: 16-bit / NHWC input needs a 16-bit 1x1 conv", fn);
  if (!m2f::aligned(dO, 16) || (i16 && !i_nhwc && !m2f::aligned(I, 16))) return m2f::fail(M2F_EINVAL, "%s: misaligned", fn);
  const int64_t M = static_cast<int64_t>(N) * H * W;
  const WgPlan p = wg_plan(M, T * Ci, Co);
  const int64_t need = static_cast<int64_t>(p.splits) * (static_cast<int64_t>(T) * Ci * Co + Co) * 4;
  if (workspace_bytes < need) return m2f::fail(M2F_EINVAL, "%s: workspace too small", fn);
  hipStream_t st = static_cast<hipStream_t>(stream);
  float* slab = static_cast<float*>(workspace);
  float* bslab = slab + static_cast<int64_t>(p.splits) * T * Ci * Co;
  const int tiles = ((T * Ci + 127) / 128) * ((Co + 255) / 256);
  const unsigned grid = static_cast<unsigned>(p.splits * tiles);
  float* bs = dbias ? bslab : nullptr;
  if (i_dtype == M2F_F32) launch_wgrad<float, false>(T, grid, dO, I, N, Co, Ci, H, W, p.rows, slab, bs, st);
  else if (i_dtype == M2F_F16 && i_nhwc) launch_wgrad<_Float16, true>(T, grid, dO, I, N, Co, Ci, H, W, p.rows, slab, bs, st);
  else if (i_dtype == M2F_F16) launch_wgrad<_Float16, false>(T, grid, dO, I, N, Co, Ci, H, W, p.rows, slab, bs, st);
  else if (i_nhwc) launch_wgrad<__bf16, true>(T, grid, dO, I, N, Co, Ci, H, W, p.rows, slab, bs, st);
  else launch_wgrad<__bf16, false>(T, grid, dO, I, N, Co, Ci, H, W, p.rows, slab, bs, st);
  if ((rc = m2f::check_launch(fn))) return rc;
  // the slab sum lands as [(tap, ci)][co]; the caller permutes it to [co][ci][tap]
  const int64_t n = static_cast<int64_t>(T) * Ci * Co;
  x3_conv_slab_reduce<<<m2f::ceil_div(n, 256), 256, 0, st>>>(slab, p.splits, n, dW);
  if ((rc = m2f::check_launch(fn))) return rc;
  if (dbias) {
    x3_conv_slab_reduce<<<m2f::ceil_div(Co, 256), 256, 0, st>>>(bslab, p.splits, Co, dbias);
    return m2f::check_launch(fn);
  }
  return m2f::ok();
}

}  // namespace

// mode 0: O = conv(I, Wt) (+ bias): I [N][Ci][H][W], O [N][Co][H][W]
// mode 1: O = conv_transpose-style input gradient of dO: I = dO [N][Co][H][W], O = dI [N][Ci][H][W]
extern "C" int m2f_conv_f32x3(const float* I, const float* Wt, const float* bias, float* O, int N, int Ci, int Co,
                              int H, int W, int ksize, int mode, void* workspace, int64_t workspace_bytes,
                              void* stream) {
  return conv_impl("m2f_conv_f32x3", I, M2F_F32, 0, Wt, bias, O, M2F_F32, 0, N, Ci, Co, H, W, ksize, mode, workspace,
                   workspace_bytes, stream);
}

extern "C" int m2f_conv_x3_io(const void* I, int i_dtype, int i_nhwc, const float* Wt, const float* bias, void* O,
                              int o_dtype, int o_nhwc, int N, int Ci, int Co, int H, int W, int ksize, int mode,
                              void* workspace, int64_t workspace_bytes, void* stream) {
  return conv_impl("m2f_conv_x3_io", I, i_dtype, i_nhwc, Wt, bias, O, o_dtype, o_nhwc, N, Ci, Co, H, W, ksize, mode,
                   workspace, workspace_bytes, stream);
}

// dW_tck [k*k][Ci][Co] = sum_{n,p} dO[n][co][p] I[n][ci][p + s(tap)]; dbias [Co] = sum dO (if dbias)
extern "C" int m2f_conv_f32x3_wgrad(const float* dO, const float* I, float* dW, float* dbias, int N, int Ci, int Co,
                                    int H, int W, int ksize, void* workspace, int64_t workspace_bytes, void* stream) {
  return wgrad_impl("m2f_conv_f32x3_wgrad", dO, I, M2F_F32, 0, dW, dbias, N, Ci, Co, H, W, ksize, workspace,
                    workspace_bytes, stream);
}

extern "C" int m2f_conv_x3_wgrad_io(const float* dO, const void* I, int i_dtype, int i_nhwc, float* dW, float* dbias,
                                    int N, int Ci, int Co, int H, int W, int ksize, void* workspace,
                                    int64_t workspace_bytes, void* stream) {
  return wgrad_impl("m2f_conv_x3_wgrad_io", dO, I, i_dtype, i_nhwc, dW, dbias, N, Ci, Co, H, W, ksize, workspace,
                    workspace_bytes, stream);
}
