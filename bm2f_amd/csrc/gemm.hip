// Exact-fp32 GEMMs for the pixel decoder's linear layers on the f32-input MFMA (v_mfma_f32_32x32x2_f32).
//
// The encoder layer (msdeformattn.py:92-131; ms_deform_attn.py value_proj / sampling_offsets /
// attention_weights / output_proj) runs five nn.Linear layers per layer on (N*S, 256) fp32 rows with
// autocast disabled (msdeformattn.py:314,320).  gfx950 has no xf32/TF32: fp32 GEMMs run at the f32
// MFMA rate (155 TF measured peak), so the kernels here are about reaching that rate on tall-skinny
// shapes (M = 344064, N and K in {256, 288, 1024}) and fusing the epilogues that otherwise cost a full
// pass over HBM each (bias, ReLU, ReLU mask, bias gradient).
//
//   gemm_nt:  C[M,N] = A[M,K] . B[N,K]^T  (+ bias[N]) (ReLU | * [mask[M,N] > 0])
//             forward (B = W) and input gradient (B = W^T, transposed once per call: <= 1 MB)
//   gemm_tn:  C[N1,N2] = A[M,N1]^T . B[M,N2]   split over M, fp32 slabs reduced in a fixed order
//             (deterministic); optionally colsum[N1] = sum_m A[m,:]  (the bias gradient)
//
// MFMA operand trick: a 32x32x2 MFMA sums over k' = lane>>5.  Feeding lane half h the values at
// k = 8*kk + 4*h + s in MFMA s = 0..3 covers k = 8*kk .. 8*kk+7 exactly once, and makes each lane's four
// A (and B) values CONTIGUOUS in k: one ds_read_b128 per fragment instead of four ds_read_b32.  The
// products are the same; only the order of the fp32 fma chain differs from a k-sequential loop.
#include "bm2f.h"
#include "common.h"

#include <hip/hip_runtime.h>

#include <cstdlib>
#include <type_traits>

namespace {

using f4 = float __attribute__((ext_vector_type(4)));
using f16v = float __attribute__((ext_vector_type(16)));

constexpr int kBM = 128, kBN = 128, kBK = 32;
constexpr int kPitch = kBK + 4;  // floats per LDS row: 144 B, conflict-free ds_read_b128 over 8 rows
constexpr int kThreads = 256;

__device__ __forceinline__ f16v mfma32(float a, float b, f16v c) {
  return __builtin_amdgcn_mfma_f32_32x32x2f32(a, b, c, 0, 0, 0);
}

// bijective XCD-aware remap: consecutive logical ids land on the same XCD (blocks id, id+8, ... share one)
__device__ __forceinline__ int xcd_remap(int id, int nwg) {
  const int q = nwg / 8, r = nwg % 8, xcd = id % 8;
  return (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + id / 8;
}

enum Epi { kNone = 0, kBias = 1, kRelu = 2, kMask = 4 };

// ---------------------------------------------------------------------------------------------------
// NT: block BM x BN, WM x WN waves, each wave TI x TJ MFMA tiles of 32x32; K step 32, LDS double buffer
// with the next tile's global loads in flight (registers) during the current tile's MFMAs.
// ---------------------------------------------------------------------------------------------------
template <int BM, int BN, int WM, int WN, int EPI, int DEPTH>
__global__ void __launch_bounds__(64 * WM * WN) gemm_nt_kernel(const float* __restrict__ A, int64_t lda,
                                                              const float* __restrict__ B, int64_t ldb,
                                                              const float* __restrict__ bias,
                                                              const float* __restrict__ mask, int64_t ldm,
                                                              float* __restrict__ C, int64_t ldc, int M, int N,
                                                              int K) {
  constexpr int NT = 64 * WM * WN;
  constexpr int TI = BM / WM / 32, TJ = BN / WN / 32;
  constexpr int NA = BM * 8 / NT, NB = BN * 8 / NT;  // float4 loads per thread per K step
  static_assert(TI * WM * 32 == BM && TJ * WN * 32 == BN, "tile");
  static_assert(NA * NT == BM * 8 && NB * NT == BN * 8, "staging");
  __shared__ __attribute__((aligned(16))) float smem[2][(BM + BN) * kPitch];  // [buf][A rows | B rows][k]
  const int nbn = (N + BN - 1) / BN;
  const int tile = xcd_remap(blockIdx.x, gridDim.x);
  const int bm = tile / nbn, bn = tile % nbn;
  const int m0 = bm * BM, n0 = bn * BN;
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const int wm = w / WN, wn = w % WN;
  const int li = lane & 31, lh = lane >> 5;

  // register staging ring of DEPTH tiles (DEPTH 1: the next tile's loads fly during one K step; DEPTH 2:
  // during two).  Slots are compile-time indices: the K loop is unrolled by DEPTH.
  f4 ra[DEPTH][NA], rb[DEPTH][NB];
  auto gload = [&](int k0, auto slot) {
    constexpr int sl = decltype(slot)::value;
#pragma unroll
    for (int u = 0; u < NA; ++u) {
      const int idx = tid + u * NT, r = idx >> 3, k = k0 + (idx & 7) * 4;
      const int gm = m0 + r;
      ra[sl][u] = (gm < M && k < K) ? *reinterpret_cast<const f4*>(A + gm * lda + k) : f4{0.f, 0.f, 0.f, 0.f};
    }
#pragma unroll
    for (int u = 0; u < NB; ++u) {
      const int idx = tid + u * NT, r = idx >> 3, k = k0 + (idx & 7) * 4;
      const int gn = n0 + r;
      rb[sl][u] = (gn < N && k < K) ? *reinterpret_cast<const f4*>(B + gn * ldb + k) : f4{0.f, 0.f, 0.f, 0.f};
    }
  };
  auto sstore = [&](int buf, auto slot) {
    constexpr int sl = decltype(slot)::value;
#pragma unroll
    for (int u = 0; u < NA; ++u) {
      const int idx = tid + u * NT;
      *reinterpret_cast<f4*>(&smem[buf][(idx >> 3) * kPitch + (idx & 7) * 4]) = ra[sl][u];
    }
#pragma unroll
    for (int u = 0; u < NB; ++u) {
      const int idx = tid + u * NT;
      *reinterpret_cast<f4*>(&smem[buf][(BM + (idx >> 3)) * kPitch + (idx & 7) * 4]) = rb[sl][u];
    }
  };

  f16v acc[TI][TJ];
#pragma unroll
  for (int i = 0; i < TI; ++i)
#pragma unroll
    for (int j = 0; j < TJ; ++j)
#pragma unroll
      for (int e = 0; e < 16; ++e) acc[i][j][e] = 0.f;

  auto compute = [&](int buf) {
    const float* sa = smem[buf];
    const float* sb = smem[buf] + BM * kPitch;
#pragma unroll
    for (int kk = 0; kk < kBK / 8; ++kk) {
      f4 fa[TI], fb[TJ];
#pragma unroll
      for (int i = 0; i < TI; ++i)
        fa[i] = *reinterpret_cast<const f4*>(&sa[(wm * TI * 32 + i * 32 + li) * kPitch + kk * 8 + lh * 4]);
#pragma unroll
      for (int j = 0; j < TJ; ++j)
        fb[j] = *reinterpret_cast<const f4*>(&sb[(wn * TJ * 32 + j * 32 + li) * kPitch + kk * 8 + lh * 4]);
#pragma unroll
      for (int s = 0; s < 4; ++s)
#pragma unroll
        for (int i = 0; i < TI; ++i)
#pragma unroll
          for (int j = 0; j < TJ; ++j) acc[i][j] = mfma32(fa[i][s], fb[j][s], acc[i][j]);
    }
  };

  using S0 = std::integral_constant<int, 0>;
  using S1 = std::integral_constant<int, DEPTH - 1>;
  const int nk = (K + kBK - 1) / kBK;
  if constexpr (DEPTH == 1) {
    gload(0, S0{});
    sstore(0, S0{});
    __syncthreads();
    for (int kt = 0; kt < nk; ++kt) {
      const int buf = kt & 1;
      if (kt + 1 < nk) gload((kt + 1) * kBK, S0{});
      compute(buf);
      if (kt + 1 < nk) sstore(buf ^ 1, S0{});
      __syncthreads();
    }
  } else {
    // tile t is staged in register slot t & 1 and LDS buffer t & 1
    gload(0, S0{});
    if (nk > 1) gload(kBK, S1{});
    sstore(0, S0{});
    __syncthreads();
    auto step = [&](int kt, auto cur, auto nxt) {
      // cur = slot of tile kt (already in LDS, free for tile kt+2); nxt = slot of tile kt+1
      if (kt + 2 < nk) gload((kt + 2) * kBK, cur);
      compute(kt & 1);
      if (kt + 1 < nk) sstore((kt + 1) & 1, nxt);
      __syncthreads();
    };
    for (int kt = 0; kt < nk; kt += 2) {
      step(kt, S0{}, S1{});
      if (kt + 1 < nk) step(kt + 1, S1{}, S0{});
    }
  }

  // epilogue through LDS: each wave drops its accumulators into a [BM][BN + 4] fp32 image (lane holds
  // C[row = (e&3) + 8*(e>>2) + 4*lh][col = li] of each 32x32 tile: 32 consecutive floats per row and
  // store instruction), then every thread streams whole rows out as float4 with the bias / ReLU / mask
  // applied -- 4x fewer memory instructions than per-element stores, and the mask read is coalesced.
  constexpr int CP = BN + 4;
  static_assert(BM * CP <= 2 * (BM + BN) * kPitch, "C image fits the staging buffers");
  float* cimg = &smem[0][0];  // the loop ended with a barrier: staging buffers are free
#pragma unroll
  for (int i = 0; i < TI; ++i)
#pragma unroll
    for (int j = 0; j < TJ; ++j)
#pragma unroll
      for (int e = 0; e < 16; ++e)
        cimg[(wm * TI * 32 + i * 32 + (e & 3) + 8 * (e >> 2) + 4 * lh) * CP + wn * TJ * 32 + j * 32 + li] = acc[i][j][e];
  __syncthreads();
  constexpr int C4 = BN / 4;  // float4 per tile row
  const bool vec_ok = ((N & 3) == 0) && ((ldc & 3) == 0) && (!(EPI & kMask) || (ldm & 3) == 0);
  for (int idx = tid; idx < BM * C4; idx += NT) {
    const int r = idx / C4, c = (idx - r * C4) * 4;
    const int row = m0 + r, col = n0 + c;
    if (row >= M || col >= N) continue;
    f4 v = *reinterpret_cast<const f4*>(&cimg[r * CP + c]);
    if (vec_ok) {
      if constexpr ((EPI & kBias) != 0) v += *reinterpret_cast<const f4*>(bias + col);
      if constexpr ((EPI & kRelu) != 0) {
        v.x = fmaxf(v.x, 0.f); v.y = fmaxf(v.y, 0.f); v.z = fmaxf(v.z, 0.f); v.w = fmaxf(v.w, 0.f);
      }
      if constexpr ((EPI & kMask) != 0) {
        const f4 mk = *reinterpret_cast<const f4*>(mask + row * ldm + col);
        v.x = mk.x > 0.f ? v.x : 0.f; v.y = mk.y > 0.f ? v.y : 0.f;
        v.z = mk.z > 0.f ? v.z : 0.f; v.w = mk.w > 0.f ? v.w : 0.f;
      }
      *reinterpret_cast<f4*>(C + row * ldc + col) = v;
    } else {
#pragma unroll
      for (int t = 0; t < 4; ++t) {
        if (col + t >= N) break;
        float x = v[t];
        if constexpr ((EPI & kBias) != 0) x += bias[col + t];
        if constexpr ((EPI & kRelu) != 0) x = fmaxf(x, 0.f);
        if constexpr ((EPI & kMask) != 0) x = mask[row * ldm + col + t] > 0.f ? x : 0.f;
        C[row * ldc + col + t] = x;
      }
    }
  }
}

template <int BM, int BN, int WM, int WN, int DEPTH = 1>
int launch_nt(int epi, const float* A, int64_t lda, const float* B, int64_t ldb, const float* bias,
              const float* mask, int64_t ldm, float* C, int64_t ldc, int M, int N, int K, hipStream_t st) {
  const int64_t nwg = static_cast<int64_t>((M + BM - 1) / BM) * ((N + BN - 1) / BN);
  if (nwg > 0x7fffffff) return m2f::fail(M2F_EUNSUPPORTED, "m2f_gemm_f32_nt: too many tiles");
  const dim3 grid(static_cast<unsigned>(nwg)), block(64 * WM * WN);
#define M2F_NT(E) gemm_nt_kernel<BM, BN, WM, WN, E, DEPTH><<<grid, block, 0, st>>>(A, lda, B, ldb, bias, mask, ldm, C, ldc, M, N, K)
  switch (epi) {
    case kNone: M2F_NT(kNone); break;
    case kBias: M2F_NT(kBias); break;
    case kRelu: M2F_NT(kRelu); break;
    case kBias | kRelu: M2F_NT(kBias | kRelu); break;
    case kMask: M2F_NT(kMask); break;
    case kBias | kMask: M2F_NT(kBias | kMask); break;
    default: return m2f::fail(M2F_EINVAL, "m2f_gemm_f32_nt: epilogue %d", epi);
  }
#undef M2F_NT
  return m2f::check_launch("m2f_gemm_f32_nt");
}

// ---------------------------------------------------------------------------------------------------
// TN split-M: C[N1,N2] partial over rows [r0, r1) per block, slab per split; 4 waves as 2x2 of 64x64.
// LDS image [k = row of A/B][n], pitch 136 floats: lanes of one half read 32 consecutive n (conflict
// free), the other half 4 rows further, 32 banks over.
// ---------------------------------------------------------------------------------------------------
constexpr int kTPitch = kBN + 8;

__global__ void __launch_bounds__(kThreads, 2) gemm_tn_kernel(const float* __restrict__ A, int64_t lda,
                                                             const float* __restrict__ B, int64_t ldb, int M, int N1,
                                                             int N2, int rows_per_split, float* __restrict__ slab,
                                                             float* __restrict__ colsum_slab) {
  __shared__ __attribute__((aligned(16))) float smem[2][2][kBK * kTPitch];  // [buf][A|B][k][n]
  const int nb1 = (N1 + kBM - 1) / kBM, nb2 = (N2 + kBN - 1) / kBN;
  const int tiles = nb1 * nb2;
  const int id = xcd_remap(blockIdx.x, gridDim.x);
  const int split = id / tiles, t = id % tiles;
  const int b1 = t / nb2, b2 = t % nb2;
  const int n10 = b1 * kBM, n20 = b2 * kBN;
  const int r0 = split * rows_per_split;
  const int r1 = min(M, r0 + rows_per_split);
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const int wm = w >> 1, wn = w & 1;
  const int li = lane & 31, lh = lane >> 5;
  const bool do_colsum = colsum_slab != nullptr && b2 == 0;

  // staging: 32 rows x 32 float4 per operand -> 4 per thread; row = idx >> 5, n4 = idx & 31
  f4 ra[4], rb[4];
  auto gload = [&](int k0) {
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      const int idx = tid + u * kThreads, r = k0 + (idx >> 5), n = (idx & 31) * 4;
      const bool rok = r < r1;
      ra[u] = (rok && n10 + n < N1) ? *reinterpret_cast<const f4*>(A + r * lda + n10 + n) : f4{0.f, 0.f, 0.f, 0.f};
      rb[u] = (rok && n20 + n < N2) ? *reinterpret_cast<const f4*>(B + r * ldb + n20 + n) : f4{0.f, 0.f, 0.f, 0.f};
    }
  };
  f4 csum = {0.f, 0.f, 0.f, 0.f};  // column sums of A for columns (tid & 31)*4 .. +3, rows tid>>5 (+8u)
  auto sstore = [&](int buf) {
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      const int idx = tid + u * kThreads, r = idx >> 5, n4 = idx & 31;
      *reinterpret_cast<f4*>(&smem[buf][0][r * kTPitch + n4 * 4]) = ra[u];
      *reinterpret_cast<f4*>(&smem[buf][1][r * kTPitch + n4 * 4]) = rb[u];
      if (do_colsum) csum += ra[u];
    }
  };

  f16v acc[2][2];
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j)
#pragma unroll
      for (int e = 0; e < 16; ++e) acc[i][j][e] = 0.f;

  const int nk = r1 > r0 ? (r1 - r0 + kBK - 1) / kBK : 0;
  if (nk > 0) {
    gload(r0);
    sstore(0);
  }
  __syncthreads();
  for (int kt = 0; kt < nk; ++kt) {
    const int buf = kt & 1;
    if (kt + 1 < nk) gload(r0 + (kt + 1) * kBK);
    const float* sa = smem[buf][0];
    const float* sb = smem[buf][1];
#pragma unroll
    for (int kk = 0; kk < kBK / 8; ++kk) {
#pragma unroll
      for (int s = 0; s < 4; ++s) {
        const int k = kk * 8 + lh * 4 + s;
        float fa[2], fb[2];
#pragma unroll
        for (int i = 0; i < 2; ++i) fa[i] = sa[k * kTPitch + wm * 64 + i * 32 + li];
#pragma unroll
        for (int j = 0; j < 2; ++j) fb[j] = sb[k * kTPitch + wn * 64 + j * 32 + li];
#pragma unroll
        for (int i = 0; i < 2; ++i)
#pragma unroll
          for (int j = 0; j < 2; ++j) acc[i][j] = mfma32(fa[i], fb[j], acc[i][j]);
      }
    }
    if (kt + 1 < nk) sstore(buf ^ 1);
    __syncthreads();
  }

  // slab[split][N1][N2]
  float* out = slab + static_cast<int64_t>(split) * N1 * N2;
#pragma unroll
  for (int j = 0; j < 2; ++j) {
    const int col = n20 + wn * 64 + j * 32 + li;
    if (col >= N2) continue;
#pragma unroll
    for (int i = 0; i < 2; ++i) {
#pragma unroll
      for (int e = 0; e < 16; ++e) {
        const int row = n10 + wm * 64 + i * 32 + (e & 3) + 8 * (e >> 2) + 4 * lh;
        if (row < N1) out[static_cast<int64_t>(row) * N2 + col] = acc[i][j][e];
      }
    }
  }
  if (do_colsum) {
    // reduce the 8 row phases (tid >> 5) of each column group through LDS (reuse buffer 0)
    float* red = smem[0][0];
    __syncthreads();
    *reinterpret_cast<f4*>(&red[(tid >> 5) * kTPitch + (tid & 31) * 4]) = csum;
    __syncthreads();
    if (tid < kBM) {
      float v = 0.f;
#pragma unroll
      for (int p = 0; p < 8; ++p) v += red[p * kTPitch + tid];
      if (n10 + tid < N1) colsum_slab[static_cast<int64_t>(split) * N1 + n10 + tid] = v;
    }
  }
}

// out[i] = sum_s slab[s][i] in split order (deterministic); 4 independent chains per thread
__global__ void __launch_bounds__(256) slab_reduce_kernel(const float* __restrict__ slab, int splits, int64_t n,
                                                          float* __restrict__ out, int64_t ldo, int ncols) {
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
  const int64_t r = i / ncols, c = i % ncols;
  out[r * ldo + c] = (a0 + a1) + (a2 + a3);
}

int tn_splits(int M, int N1, int N2) {
  const int tiles = ((N1 + kBM - 1) / kBM) * ((N2 + kBN - 1) / kBN);
  int splits = (1024 + tiles - 1) / tiles;                     // ~1024 blocks: 2 per CU, 2 rounds
  const int max_splits = (M + 4 * kBK - 1) / (4 * kBK);         // >= 4 K-steps per block
  if (splits > max_splits) splits = max_splits;
  return splits < 1 ? 1 : splits;
}

int tn_rows_per_split(int M, int splits) {
  const int r = (M + splits - 1) / splits;
  return (r + kBK - 1) / kBK * kBK;
}

}  // namespace

extern "C" int m2f_gemm_f32_nt(const float* A, int64_t lda, const float* B, int64_t ldb, const float* bias,
                               int relu, const float* mask, int64_t ldm, float* C, int64_t ldc, int M, int N, int K,
                               void* stream) {
  const char* fn = "m2f_gemm_f32_nt";
  if (M < 0 || N <= 0 || K <= 0) return m2f::fail(M2F_EINVAL, "%s: M %d N %d K %d", fn, M, N, K);
  if (!A || !B || !C) return m2f::fail(M2F_EINVAL, "%s: null pointer", fn);
  if (K % 4 || lda % 4 || ldb % 4 || lda < K || ldb < K || ldc < N || !m2f::aligned(A, 16) || !m2f::aligned(B, 16))
    return m2f::fail(M2F_EINVAL, "%s: K, lda, ldb must be multiples of 4 (>= K), A/B 16-byte aligned", fn);
  if (mask && ldm < N) return m2f::fail(M2F_EINVAL, "%s: ldm %lld < N", fn, static_cast<long long>(ldm));
  if (relu && mask) return m2f::fail(M2F_EINVAL, "%s: relu and mask are exclusive", fn);
  if (M == 0) return m2f::ok();
  hipStream_t st = static_cast<hipStream_t>(stream);
  const int epi = (bias ? kBias : 0) | (relu ? kRelu : 0) | (mask ? kMask : 0);
  // tile choice: N a multiple of 96 but not 128 (the 288-wide sampling projection) gets 96-wide blocks
  int cfg = (N % 128 != 0 && N % 96 == 0) ? 4 : 0;
  cfg = m2f::option(m2f::kOptGemmNtCfg, cfg);
  switch (cfg) {
    case 0: return launch_nt<128, 128, 2, 2>(epi, A, lda, B, ldb, bias, mask, ldm, C, ldc, M, N, K, st);
    case 4: return launch_nt<128, 96, 4, 1>(epi, A, lda, B, ldb, bias, mask, ldm, C, ldc, M, N, K, st);
    case 6: return launch_nt<128, 128, 4, 1>(epi, A, lda, B, ldb, bias, mask, ldm, C, ldc, M, N, K, st);
    case 7: return launch_nt<128, 128, 4, 1, 2>(epi, A, lda, B, ldb, bias, mask, ldm, C, ldc, M, N, K, st);
    case 8: return launch_nt<128, 96, 4, 1, 2>(epi, A, lda, B, ldb, bias, mask, ldm, C, ldc, M, N, K, st);
    case 9: return launch_nt<128, 128, 2, 2, 2>(epi, A, lda, B, ldb, bias, mask, ldm, C, ldc, M, N, K, st);
    default: return m2f::fail(M2F_EINVAL, "%s: config %d", fn, cfg);
  }
}

extern "C" int m2f_gemm_f32_tn_workspace(int M, int N1, int N2, int64_t* workspace_bytes) {
  if (M < 0 || N1 <= 0 || N2 <= 0) return m2f::fail(M2F_EINVAL, "m2f_gemm_f32_tn_workspace: bad sizes");
  const int splits = tn_splits(M, N1, N2);
  if (workspace_bytes) *workspace_bytes = static_cast<int64_t>(splits) * (static_cast<int64_t>(N1) * N2 + N1) * 4;
  return m2f::ok();
}

extern "C" int m2f_gemm_f32_tn(const float* A, int64_t lda, const float* B, int64_t ldb, float* C, int64_t ldc,
                               float* colsum, int M, int N1, int N2, void* workspace, int64_t workspace_bytes,
                               void* stream) {
  const char* fn = "m2f_gemm_f32_tn";
  if (M < 0 || N1 <= 0 || N2 <= 0) return m2f::fail(M2F_EINVAL, "%s: M %d N1 %d N2 %d", fn, M, N1, N2);
  if ((M > 0 && (!A || !B)) || !C) return m2f::fail(M2F_EINVAL, "%s: null pointer", fn);  // M = 0: C = 0
  if (N1 % 4 || N2 % 4 || lda % 4 || ldb % 4 || lda < N1 || ldb < N2 || ldc < N2 || !m2f::aligned(A, 16) ||
      !m2f::aligned(B, 16))
    return m2f::fail(M2F_EINVAL, "%s: N1, N2, lda, ldb must be multiples of 4, A/B 16-byte aligned", fn);
  const int splits = tn_splits(M, N1, N2);
  const int64_t need = static_cast<int64_t>(splits) * (static_cast<int64_t>(N1) * N2 + N1) * 4;
  if (!workspace || workspace_bytes < need)
    return m2f::fail(M2F_EINVAL, "%s: workspace %lld < %lld", fn, static_cast<long long>(workspace_bytes),
                     static_cast<long long>(need));
  hipStream_t st = static_cast<hipStream_t>(stream);
  float* slab = static_cast<float*>(workspace);
  float* cslab = slab + static_cast<int64_t>(splits) * N1 * N2;
  const int tiles = ((N1 + kBM - 1) / kBM) * ((N2 + kBN - 1) / kBN);
  const int rps = tn_rows_per_split(M, splits);
  gemm_tn_kernel<<<splits * tiles, kThreads, 0, st>>>(A, lda, B, ldb, M, N1, N2, rps, slab, colsum ? cslab : nullptr);
  if (int rc = m2f::check_launch(fn)) return rc;
  const int64_t n = static_cast<int64_t>(N1) * N2;
  slab_reduce_kernel<<<m2f::ceil_div(n, 256), 256, 0, st>>>(slab, splits, n, C, ldc, N2);
  if (int rc = m2f::check_launch(fn)) return rc;
  if (colsum) {
    slab_reduce_kernel<<<m2f::ceil_div(N1, 256), 256, 0, st>>>(cslab, splits, N1, colsum, N1, N1);
    return m2f::check_launch(fn);
  }
  return m2f::ok();
}
