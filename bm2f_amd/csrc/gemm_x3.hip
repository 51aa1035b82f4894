// fp32 GEMMs on the bf16 matrix cores by exact three-way operand splitting ("x3" GEMMs).
//
// The pixel decoder's encoder linears run in fp32 (msdeformattn.py:314,320 force autocast off).  gfx950
// has no xf32/TF32 and its f32-input MFMA runs at 1/16 of the bf16 rate (MI355X_MICROARCH.md, matrix
// cores), so the exact-f32 kernels of gemm.hip top out at ~157 TF.  Here every fp32 operand is split
// into three bf16 planes
//
//     x = h + m + l,   h = bf16(x),  m = bf16(x - h),  l = bf16(x - h - m)
//
// (each subtraction is exact in fp32; h, m, l carry 8 significant bits each, so x - h - m - l is at most
// 2^-24 |x|: the split is fp32-exact up to the last bit).  A product is then the six bf16 MFMA terms of
// order <= 2^-16,
//
//     a.b ~ ah.bh + ah.bm + am.bh + ah.bl + am.bm + al.bh
//
// dropping am.bl + al.bm + al.bl (<= ~2^-24 |a||b|, the size of one fp32 rounding).  bf16 x bf16 products
// are exact in fp32 and the MFMA accumulates in fp32, so the result is an fp32-accurate GEMM (error vs an
// fp64 reference at the level of the exact-f32 MFMA kernels; tests/test_gemm_x3_gpu.py pins it) at
// 16/6 = 2.7x the f32 MFMA peak.  This is an fp32 GEMM, not a reduced-precision one: no input bit that
// fp32 keeps is dropped.  Non-finite inputs keep their fp32 meaning (h = x, m = l = 0).
//
//   x3_nt:  C[M,N] = A[M,K] . B[N,K]^T  (+ bias[N]) (ReLU | * [mask[M,N] > 0])        forward, dgrad
//   x3_tn:  C[N1,N2] = A[M,N1]^T . B[M,N2] over M-slabs, reduced in a fixed order;   wgrad (+ bias grad)
//           optionally colsum[N1] = sum_m A[m,:]
//
// Both kernels share one LDS image per stage: for each operand and plane, rows (M/N1 rows for A, N/N2
// rows for B) of BK = 16 bf16 along k with a 48-byte pitch, so the 32x32x16 operand read of a lane
// (row l&31, k 8(l>>5) .. +7) is one conflict-free ds_read_b128.  NT stages rows as they lie in memory;
// TN transposes while splitting (a thread owns one column and 8 consecutive k).  Double-buffered, one
// barrier per k-step, the next step's global loads in flight during the MFMAs.
#include "bm2f.h"
#include "common.h"
#include "x3_device.h"

#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdlib>

namespace {

using namespace m2f_x3;

// kAdd: C = A.B (+bias) + D1 (+ D2);  kBitsOut: with kRelu, also bits[m][n / 32] bit n % 32 = (C > 0) (the FFN's
// ReLU mask, 1 bit per element);  kBitsIn: C = A.B masked by those bits (the FFN input gradient's ReLU backward)
enum Epi { kNone = 0, kBias = 1, kRelu = 2, kMask = 4, kAdd = 8, kBitsOut = 16, kBitsIn = 32 };

// bit t of each of the four bytes -> bits 4 j + t of a word (j = byte index): the 8 lanes x 4 columns of one
// epilogue row, ballot-gathered per column offset t, become that row's 32-column mask word
__device__ __forceinline__ unsigned spread4(unsigned byte) {
  unsigned x = byte & 0xffu;
  x = (x | (x << 12)) & 0x000F000Fu;
  x = (x | (x << 6)) & 0x03030303u;
  x = (x | (x << 3)) & 0x11111111u;
  return x;
}

// ---------------------------------------------------------------------------------------------------
// NT: C[M,N] = A[M,K] . B[N,K]^T.
//
// B (a weight: <= 1024 x 1024) is split once per call into planes Bs[k16 chunk][plane][NP][16] bf16
// (x3_presplit; NP = N rounded up to the block width, zero-filled).  Rows are 32 B with the two 16-B
// halves swapped on rows whose bit 3 is set: with that swizzle the dense image is conflict-free for the
// 32x32x16 operand read (ds_read_b128 lane groups {0-3,12-15,20-27}, ... cover all 64 banks once), so a
// chunk is copied to LDS as one linear 16-byte-per-thread stream.
//
// A block of NW waves owns NW*32 rows of A and BN columns of C; each wave owns 32 rows.  A wave loads its
// own A fragments straight from HBM into registers (lane (r, h): row r, k 8h .. 8h+7 of the chunk, two
// float4), splits them in registers, and multiplies them against the block's B chunk in LDS.  A never
// touches LDS and is split once.  Pipeline: global loads run two chunks ahead in two register sets (the
// loop is unrolled by 2 so the sets are static); chunk c+1 is written to the other LDS buffer and split
// while chunk c's MFMAs drain; one barrier per chunk.
// Epilogue: each 32x32 accumulator tile goes through a per-wave LDS image and leaves as float4 rows, with
// the bias / ReLU / ReLU-mask applied on the way (mask reads coalesced like the stores).
// ---------------------------------------------------------------------------------------------------

__global__ void __launch_bounds__(256) x3_presplit(const float* __restrict__ B, int64_t ldb, int b_kn, int N, int K,
                                                   int NP, int nchunks, __bf16* __restrict__ Bs) {
  const int64_t t = blockIdx.x * static_cast<int64_t>(blockDim.x) + threadIdx.x;
  if (t >= static_cast<int64_t>(nchunks) * NP) return;
  const int c = static_cast<int>(t / NP), n = static_cast<int>(t - static_cast<int64_t>(c) * NP);
  bf8 pl[3][2];
#pragma unroll
  for (int j = 0; j < 16; ++j) {
    const int k = c * 16 + j;
    float v = 0.f;
    if (n < N && k < K) v = b_kn ? B[static_cast<int64_t>(k) * ldb + n] : B[static_cast<int64_t>(n) * ldb + k];
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

template <int BN, int NW, int EPI, bool KFULL>
__global__ void __launch_bounds__(64 * NW, 2) x3_nt_kernel(const float* __restrict__ A, int64_t lda,
                                                       const __bf16* __restrict__ Bs, int NP,
                                                       const float* __restrict__ bias,
                                                       const float* __restrict__ mask, int64_t ldm,
                                                       const float* D1, const float* D2, int64_t ldd, int dper,
                                                       uint32_t* bits, float* C, int64_t ldc, int M, int N, int K) {
  constexpr int NT = 64 * NW, BM = 32 * NW, TJ = BN / 32;
  constexpr int PIECES = 3 * BN * 2;             // 16-byte pieces of one B chunk
  constexpr int NBL = (PIECES + NT - 1) / NT;    // per thread
  constexpr int CHUNK = 3 * BN * 16;             // bf16 per LDS chunk image
  constexpr int EP = 36;                         // epilogue image pitch (floats)
  constexpr int LDS_B = 2 * CHUNK * 2, LDS_E = NW * 32 * EP * 4;
  __shared__ __attribute__((aligned(16))) char smem[LDS_B > LDS_E ? LDS_B : LDS_E];
  __bf16(*sb)[CHUNK] = reinterpret_cast<__bf16(*)[CHUNK]>(smem);

  const int nbn = (N + BN - 1) / BN;
  const int tile = xcd_remap(blockIdx.x, gridDim.x);
  const int bm = tile / nbn, bn = tile % nbn;
  const int m0 = bm * BM, n0 = bn * BN;
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const int li = lane & 31, lh = lane >> 5;
  const int arow = m0 + w * 32 + li;
  const float* ap = A + static_cast<int64_t>(min(arow, M - 1)) * lda + lh * 8;
  const bool arow_ok = arow < M;
  const int nk = (K + kBK - 1) / kBK;

  struct Regs {
    f4 a[2];
    bf8 b[NBL];
  };
  // branch-free: out-of-range A reads are clamped in-bounds (rows >= M only feed rows never stored; k >= K
  // is zeroed when the chunk is split, not here, so the load is not waited on early)
  auto gload = [&](Regs& r, int c) {
    const int k = c * kBK + lh * 8;
    const int cc = min(c, nk - 1);
    r.a[0] = *reinterpret_cast<const f4*>(ap + min(k, K - 4) - lh * 8);
    r.a[1] = *reinterpret_cast<const f4*>(ap + min(k + 4, K - 4) - lh * 8);
    const __bf16* bc = Bs + static_cast<int64_t>(cc) * 3 * NP * 16;
#pragma unroll
    for (int u = 0; u < NBL; ++u) {
      const int q = min(tid + u * NT, PIECES - 1);
      const int p = q / (BN * 2), rem = q - p * BN * 2;
      r.b[u] = *reinterpret_cast<const bf8*>(bc + (static_cast<int64_t>(p) * NP + n0) * 16 + rem * 8);
    }
  };
  auto bstore = [&](const Regs& r, int buf) {
#pragma unroll
    for (int u = 0; u < NBL; ++u) {
      const int q = tid + u * NT;
      if (PIECES % NT != 0 && q >= PIECES) continue;
      *reinterpret_cast<bf8*>(&sb[buf][q * 8]) = r.b[u];
    }
  };
  auto asplit = [&](const Regs& r, int c, bf8 (&fa)[3]) {
    const int k = c * kBK + lh * 8;
    float x[8];
#pragma unroll
    for (int e = 0; e < 8; ++e) x[e] = KFULL || k + e < K ? r.a[e >> 2][e & 3] : 0.f;
    split8(x, fa);
  };

  f16v acc[TJ];
#pragma unroll
  for (int j = 0; j < TJ; ++j)
#pragma unroll
    for (int e = 0; e < 16; ++e) acc[j][e] = 0.f;

  // B operand read of tile j: row j*32 + li, half lh (swizzled)
  const int boff = li * 16 + ((lh ^ swz(li)) * 8);
  auto chunk_mfma = [&](int buf, const bf8 (&fa)[3]) {
    const __bf16* base = &sb[buf][0];
#pragma unroll
    for (int j = 0; j < TJ; ++j) {
      const int off = j * 32 * 16 + boff;
      const bf8 bh = *reinterpret_cast<const bf8*>(base + off);
      const bf8 bmv = *reinterpret_cast<const bf8*>(base + BN * 16 + off);
      const bf8 bl = *reinterpret_cast<const bf8*>(base + 2 * BN * 16 + off);
      f16v x = acc[j];
      x = mfma(fa[2], bh, x);   // al.bh
      x = mfma(fa[1], bmv, x);  // am.bm
      x = mfma(fa[0], bl, x);   // ah.bl
      x = mfma(fa[1], bh, x);   // am.bh
      x = mfma(fa[0], bmv, x);  // ah.bm
      x = mfma(fa[0], bh, x);   // ah.bh
      acc[j] = x;
    }
  };

  // Pipeline: global loads two chunks ahead in two register sets (unrolled by 2 so the sets are static);
  // chunk c+1 is written to the other LDS buffer and split into the other fragment set while chunk c's
  // MFMAs drain; one barrier per chunk.  Branch-free (past the end the loads are clamped to the last chunk
  // and the stores go to the buffer no one reads again), so the split can interleave with the MFMAs
  // (a three-deep ring measured slower: 217 VGPRs).
  Regs r0, r1;
  bf8 fa[3], fb[3];
  gload(r0, 0);
  gload(r1, 1);
  bstore(r0, 0);
  asplit(r0, 0, fa);
  __syncthreads();
  auto step = [&](int c, Regs& cur, const Regs& nxt, const bf8 (&fc)[3], bf8 (&fn)[3]) {
    gload(cur, c + 2);
    M2F_X3_PREFETCH_FENCE();
    chunk_mfma(c & 1, fc);
    bstore(nxt, (c + 1) & 1);
    asplit(nxt, c + 1, fn);
    __syncthreads();
  };
  // (hipcc sinks the split of a pair's second chunk into the conditional second step, next to its MFMAs;
  // unconditional pairs with the split kept before the barrier, with or without sched_group_barrier
  // interleaving, measured 3-11 % slower here -- the opposite of the TN kernel below, r2am)
  for (int c = 0; c < nk; c += 2) {
    step(c, r0, r1, fa, fb);
    if (c + 1 < nk) step(c + 1, r1, r0, fb, fa);
  }

  // ---- epilogue -----------------------------------------------------------------------------------
  float* img = reinterpret_cast<float*>(smem) + w * 32 * EP;
  const int er = lane >> 3, ec = (lane & 7) * 4;  // read-back: 8 rows x 8 float4 per instruction
#pragma unroll
  for (int j = 0; j < TJ; ++j) {
#pragma unroll
    for (int e = 0; e < 16; ++e) img[((e & 3) + 8 * (e >> 2) + 4 * lh) * EP + li] = acc[j][e];
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    const int col = n0 + j * 32 + ec;
    f4 bv = {0.f, 0.f, 0.f, 0.f};
    if constexpr ((EPI & kBias) != 0) {
      if (col + 3 < N) bv = *reinterpret_cast<const f4*>(bias + col);
      else
        for (int t = 0; t < 4; ++t) bv[t] = col + t < N ? bias[col + t] : 0.f;
    }
    const bool vec = col + 3 < N && ((ldc & 3) == 0) && (!(EPI & kMask) || (ldm & 3) == 0);
    // the 4 row groups' epilogue operands (residual rows, mask rows, ReLU bit words), all loaded before any is used:
    // loaded inside the row loop (behind its range test), each had been a memory round trip of its own
    f4 d1v[4], d2v[4], mkv[4];
    unsigned nibv[4];
    if constexpr ((EPI & (kAdd | kMask | kBitsIn)) != 0) {
#pragma unroll
      for (int rr = 0; rr < 4; ++rr) {
        const int rowc = min(m0 + w * 32 + rr * 8 + er, M - 1);
        if constexpr ((EPI & kBitsIn) != 0)
          nibv[rr] = bits[static_cast<int64_t>(rowc) * ldm + min((n0 + j * 32) >> 5, (N - 1) >> 5)] >> ec;
        if (vec) {
          if constexpr ((EPI & kMask) != 0) mkv[rr] = *reinterpret_cast<const f4*>(mask + static_cast<int64_t>(rowc) * ldm + col);
          if constexpr ((EPI & kAdd) != 0) {
            d1v[rr] = *reinterpret_cast<const f4*>(D1 + static_cast<int64_t>(dper ? rowc % dper : rowc) * ldd + col);
            if (D2) d2v[rr] = *reinterpret_cast<const f4*>(D2 + static_cast<int64_t>(rowc) * ldd + col);
          }
        }
      }
    }
#pragma unroll
    for (int rr = 0; rr < 4; ++rr) {
      const int lr = rr * 8 + er, row = m0 + w * 32 + lr;
      f4 v = *reinterpret_cast<const f4*>(&img[lr * EP + ec]) + bv;
      if constexpr ((EPI & kRelu) != 0) {
        v.x = fmaxf(v.x, 0.f); v.y = fmaxf(v.y, 0.f); v.z = fmaxf(v.z, 0.f); v.w = fmaxf(v.w, 0.f);
      }
      if constexpr ((EPI & kBitsOut) != 0) {  // N % 32 == 0: a tile is in range or out as a whole
        const bool in = row < M && col < N;
        const unsigned long long b0 = __ballot(in && v.x > 0.f), b1 = __ballot(in && v.y > 0.f);
        const unsigned long long b2 = __ballot(in && v.z > 0.f), b3 = __ballot(in && v.w > 0.f);
        if ((lane & 7) == 0 && in) {
          const int sh = 8 * er;
          bits[static_cast<int64_t>(row) * ldm + ((n0 + j * 32) >> 5)] =
              spread4(static_cast<unsigned>(b0 >> sh)) | (spread4(static_cast<unsigned>(b1 >> sh)) << 1) |
              (spread4(static_cast<unsigned>(b2 >> sh)) << 2) | (spread4(static_cast<unsigned>(b3 >> sh)) << 3);
        }
      }
      if (row >= M || col >= N) continue;
      if constexpr ((EPI & kBitsIn) != 0) {
        const unsigned nib = nibv[rr];
        v.x = (nib & 1u) ? v.x : 0.f; v.y = (nib & 2u) ? v.y : 0.f;
        v.z = (nib & 4u) ? v.z : 0.f; v.w = (nib & 8u) ? v.w : 0.f;
      }
      if (vec) {
        if constexpr ((EPI & kMask) != 0) {
          const f4 mk = mkv[rr];
          v.x = mk.x > 0.f ? v.x : 0.f; v.y = mk.y > 0.f ? v.y : 0.f;
          v.z = mk.z > 0.f ? v.z : 0.f; v.w = mk.w > 0.f ? v.w : 0.f;
        }
        if constexpr ((EPI & kAdd) != 0) {
          // (A.B + bias) + D1 + D2, left to right: the sum autograd would form, one rounding per add
          v = v + d1v[rr];
          if (D2) v = v + d2v[rr];
        }
        *reinterpret_cast<f4*>(C + static_cast<int64_t>(row) * ldc + col) = v;
      } else {
        for (int t = 0; t < 4 && col + t < N; ++t) {
          float x = v[t];
          if constexpr ((EPI & kMask) != 0) x = mask[static_cast<int64_t>(row) * ldm + col + t] > 0.f ? x : 0.f;
          if constexpr ((EPI & kAdd) != 0) {
            x += D1[static_cast<int64_t>(dper ? row % dper : row) * ldd + col + t];
            if (D2) x += D2[static_cast<int64_t>(row) * ldd + col + t];
          }
          C[static_cast<int64_t>(row) * ldc + col + t] = x;
        }
      }
    }
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
  }
}

template <int BN, int NW>
int launch_nt(int epi, const float* A, int64_t lda, const __bf16* Bs, int NP, const float* bias, const float* mask,
              int64_t ldm, const float* D1, const float* D2, int64_t ldd, int dper, uint32_t* bits, float* C,
              int64_t ldc, int M, int N, int K, hipStream_t st) {
  constexpr int BM = 32 * NW;
  const int64_t nwg = static_cast<int64_t>((M + BM - 1) / BM) * ((N + BN - 1) / BN);
  if (nwg > 0x7fffffff) return m2f::fail(M2F_EUNSUPPORTED, "m2f_gemm_f32x3_nt: too many tiles");
  const dim3 grid(static_cast<unsigned>(nwg)), block(64 * NW);
#define M2F_X3NT(E)                                                                                            \
  (K % kBK == 0 ? x3_nt_kernel<BN, NW, E, true><<<grid, block, 0, st>>>(A, lda, Bs, NP, bias, mask, ldm, D1, D2, ldd, \
                                                                       dper, bits, C, ldc, M, N, K)               \
                : x3_nt_kernel<BN, NW, E, false><<<grid, block, 0, st>>>(A, lda, Bs, NP, bias, mask, ldm, D1, D2,     \
                                                                        ldd, dper, bits, C, ldc, M, N, K))
  switch (epi) {
    case kNone: M2F_X3NT(kNone); break;
    case kBias: M2F_X3NT(kBias); break;
    case kRelu: M2F_X3NT(kRelu); break;
    case kBias | kRelu: M2F_X3NT(kBias | kRelu); break;
    case kMask: M2F_X3NT(kMask); break;
    case kBias | kMask: M2F_X3NT(kBias | kMask); break;
    case kAdd: M2F_X3NT(kAdd); break;
    case kBias | kAdd: M2F_X3NT(kBias | kAdd); break;
    case kRelu | kBitsOut: M2F_X3NT(kRelu | kBitsOut); break;
    case kBias | kRelu | kBitsOut: M2F_X3NT(kBias | kRelu | kBitsOut); break;
    case kBitsIn: M2F_X3NT(kBitsIn); break;
    case kBias | kBitsIn: M2F_X3NT(kBias | kBitsIn); break;
    default: return m2f::fail(M2F_EINVAL, "m2f_gemm_f32x3_nt: epilogue %d", epi);
  }
#undef M2F_X3NT
  return m2f::check_launch("m2f_gemm_f32x3_nt");
}

// padded B width for a block width; every config's NP is a multiple of 384 = lcm(96, 128) so one
// workspace size serves them all
int64_t nt_np(int N) { return (N + 383) / 384 * 384; }

int64_t nt_workspace(int N, int K) {
  const int64_t nchunks = (K + kBK - 1) / kBK;
  return nchunks * 3 * nt_np(N) * 16 * 2;
}

// ---------------------------------------------------------------------------------------------------
// TN split-M: C[N1,N2] = sum over m of A[m,n1] B[m,n2], rows m split over workgroups (slabs reduced in a
// fixed order afterwards: deterministic).  The orientation is chosen so the wider operand is A.
//
// A block of NW waves owns NW*32 columns of A (rows of C) and 256 columns of B for one M-slab.  Each wave
// loads its own A^T fragments straight from HBM into registers (lane (r, h): column r, rows 8h .. 8h+7 of
// the chunk -- eight 4-byte loads, each instruction two 128-byte row segments), splits them there and
// keeps its 32 C rows x 256 C columns in accumulators.  The block's B chunk (16 rows x 256 columns) is
// split once while being transposed into the dense swizzled LDS image of the NT kernel (a thread owns one
// column x 8 rows: one 16-byte store per plane).  Two-deep register prefetch, one barrier per chunk.
// C tiles leave through a per-wave LDS image as float4 rows (transposed when the operands were swapped).
// ---------------------------------------------------------------------------------------------------
template <int NW, bool MFULL, int CSUM>   // MFULL: every chunk is 16 full rows; CSUM: 0 none, 1 of A, 2 of B
__global__ void __launch_bounds__(64 * NW, NW >= 8 ? 1 : 2) x3_tn_kernel(const float* __restrict__ A, int64_t lda,
                                                           const float* __restrict__ B, int64_t ldb, int M, int N1,
                                                           int N2, int rows_per_split, int trans_out,
                                                           float* __restrict__ slab, float* __restrict__ colsum_slab,
                                                           int colsum_b) {
  constexpr int NT = 64 * NW, BN = 256, TJ = BN / 32;
  constexpr int JOBS = BN * 2;                       // (B column, 8-row half) per chunk
  constexpr int NJ = (JOBS + NT - 1) / NT;
  constexpr int CHUNK = 3 * BN * 16;                 // bf16 per LDS image
  constexpr int EP = 36;
  constexpr int LDS_B = 2 * CHUNK * 2, LDS_E = NW * 32 * EP * 4;
  __shared__ __attribute__((aligned(16))) char smem[LDS_B > LDS_E ? LDS_B : LDS_E];
  __bf16(*sb)[CHUNK] = reinterpret_cast<__bf16(*)[CHUNK]>(smem);

  const int nb1 = (N1 + 32 * NW - 1) / (32 * NW), nb2 = (N2 + BN - 1) / BN;
  const int tiles = nb1 * nb2;
  const int id = xcd_remap(blockIdx.x, gridDim.x);
  const int split = id / tiles, t = id % tiles;
  const int b1 = t / nb2, b2 = t % nb2;
  const int n10 = b1 * 32 * NW, n20 = b2 * BN;
  const int r0 = split * rows_per_split;
  const int r1 = min(M, r0 + rows_per_split);
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const int li = lane & 31, lh = lane >> 5;
  const int acol = min(n10 + w * 32 + li, N1 - 1);
  const float* ap = A + acol;
  const int nk = r1 > r0 ? (r1 - r0 + kBK - 1) / kBK : 0;
  const bool csum_a = CSUM == 1 && b2 == 0;
  const bool csum_b = CSUM == 2 && b1 == 0;

  struct Regs {
    float a[8];
    float b[NJ][8];
  };
  // rows >= r1 are clamped in-bounds here and zeroed when split (never waited on at the load).  MFULL: the
  // chunk's first row is clamped instead (a chunk past the slab's end is never multiplied), so every load
  // is a wave-uniform row base (SGPRs) plus a per-lane 32-bit offset fixed for the kernel plus the
  // wave-uniform e * ld: one VALU add per load instead of a clamped 64-bit multiply-add
  const uint32_t aoff = static_cast<uint32_t>(lh * 8 * lda + acol);
  uint32_t boff8[NJ];
#pragma unroll
  for (int u = 0; u < NJ; ++u) {
    const int job = min(tid + u * NT, JOBS - 1), half = job / BN, col = min(n20 + job % BN, N2 - 1);
    boff8[u] = static_cast<uint32_t>(half * 8 * ldb + col);
  }
  auto gload = [&](Regs& r, int c) {
    const int m = r0 + c * kBK;
    if constexpr (MFULL) {
      const int64_t mb = min(m, M - kBK);
      const float* arow = A + mb * lda;
      const float* brow = B + mb * ldb;
#pragma unroll
      for (int e = 0; e < 8; ++e) r.a[e] = arow[aoff + static_cast<uint32_t>(e * lda)];
#pragma unroll
      for (int u = 0; u < NJ; ++u)
#pragma unroll
        for (int e = 0; e < 8; ++e) r.b[u][e] = brow[boff8[u] + static_cast<uint32_t>(e * ldb)];
    } else {
#pragma unroll
      for (int e = 0; e < 8; ++e) r.a[e] = ap[static_cast<int64_t>(min(m + lh * 8 + e, M - 1)) * lda];
#pragma unroll
      for (int u = 0; u < NJ; ++u) {
        const int job = min(tid + u * NT, JOBS - 1), half = job / BN, col = min(n20 + job % BN, N2 - 1);
#pragma unroll
        for (int e = 0; e < 8; ++e) r.b[u][e] = B[static_cast<int64_t>(min(m + half * 8 + e, M - 1)) * ldb + col];
      }
    }
  };
  float csa = 0.f, csb[NJ];
#pragma unroll
  for (int u = 0; u < NJ; ++u) csb[u] = 0.f;
  auto bstore = [&](const Regs& r, int c, int buf) {
    const int m = r0 + c * kBK;
#pragma unroll
    for (int u = 0; u < NJ; ++u) {
      const int job = tid + u * NT;
      if (JOBS % NT != 0 && job >= JOBS) continue;
      const int half = job / BN, col = job % BN;
      float v[8];
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        v[e] = MFULL || m + half * 8 + e < r1 ? r.b[u][e] : 0.f;
        if constexpr (CSUM == 2) csb[u] += csum_b && c < nk ? v[e] : 0.f;
      }
      bf8 pl[3];
      split8(v, pl);
      const int off = col * 16 + ((half ^ swz(col)) * 8);
      *reinterpret_cast<bf8*>(&sb[buf][off]) = pl[0];
      *reinterpret_cast<bf8*>(&sb[buf][BN * 16 + off]) = pl[1];
      *reinterpret_cast<bf8*>(&sb[buf][2 * BN * 16 + off]) = pl[2];
    }
  };
  auto asplit = [&](const Regs& r, int c, bf8 (&fa)[3]) {
    const int m = r0 + c * kBK + lh * 8;
    float v[8];
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      v[e] = MFULL || m + e < r1 ? r.a[e] : 0.f;
      if constexpr (CSUM == 1) csa += csum_a && c < nk ? v[e] : 0.f;
    }
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
      const bf8 bh = *reinterpret_cast<const bf8*>(base + off);
      const bf8 bmv = *reinterpret_cast<const bf8*>(base + BN * 16 + off);
      const bf8 bl = *reinterpret_cast<const bf8*>(base + 2 * BN * 16 + off);
      f16v x = acc[j];
      x = mfma(fa[2], bh, x);   // al.bh
      x = mfma(fa[1], bmv, x);  // am.bm
      x = mfma(fa[0], bl, x);   // ah.bl
      x = mfma(fa[1], bh, x);   // am.bh
      x = mfma(fa[0], bmv, x);  // ah.bm
      x = mfma(fa[0], bh, x);   // ah.bh
      acc[j] = x;
    }
  };

  if (nk > 0) {
    // as the NT pipeline: branch-free steps with two fragment sets.  Past the slab's end the loads are
    // clamped in-bounds and the rows zeroed (m >= r1), so the extra chunk a step splits contributes nothing
    // and its colsum terms are 0; its stores go to the buffer no one reads again.
    Regs r0s, r1s;
    bf8 fa[3], fb[3];
    gload(r0s, 0);
    gload(r1s, 1);
    bstore(r0s, 0, 0);
    asplit(r0s, 0, fa);
    __syncthreads();
    auto step = [&](int c, Regs& cur, const Regs& nxt, const bf8 (&fc)[3], bf8 (&fn)[3]) {
      gload(cur, c + 2);
      M2F_X3_PREFETCH_FENCE();
      chunk_mfma(c & 1, fc);
      bstore(nxt, c + 1, (c + 1) & 1);
      asplit(nxt, c + 1, fn);
      // keep the splits of the next chunk on this side of the barrier (hipcc otherwise moves them past it,
      // next to their MFMAs): -3..-7 % at the encoder shapes (r2am; a sched_group_barrier MFMA/VALU
      // interleave on top measured worse)
      __builtin_amdgcn_sched_barrier(0);
      __syncthreads();
    };
    // both steps of a pair unconditional, the odd last chunk peeled: a conditional second step would let
    // hipcc sink the pair's second split into it
    int c = 0;
    for (; c + 1 < nk; c += 2) {
      step(c, r0s, r1s, fa, fb);
      step(c + 1, r1s, r0s, fb, fa);
    }
    if (c < nk) step(c, r0s, r1s, fa, fb);
  }

  // ---- epilogue: slab[split] is [N1][N2] (or [N2][N1] when trans_out) --------------------------------
  const int R = trans_out ? N2 : N1, Cn = trans_out ? N1 : N2;
  float* out = slab + static_cast<int64_t>(split) * N1 * N2;
  float* img = reinterpret_cast<float*>(smem) + w * 32 * EP;
  const int er = lane >> 3, ec = (lane & 7) * 4;
#pragma unroll
  for (int j = 0; j < TJ; ++j) {
#pragma unroll
    for (int e = 0; e < 16; ++e) {
      const int rr = (e & 3) + 8 * (e >> 2) + 4 * lh;   // C row (n1) within the tile; column = li (n2)
      if (trans_out) img[li * EP + rr] = acc[j][e];
      else img[rr * EP + li] = acc[j][e];
    }
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    // image rows: n1 (normal) or n2 (transposed); columns the other index
    const int row0 = trans_out ? n20 + j * 32 : n10 + w * 32;
    const int col0 = trans_out ? n10 + w * 32 : n20 + j * 32;
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const int lr = q * 8 + er, row = row0 + lr, col = col0 + ec;
      const f4 v = *reinterpret_cast<const f4*>(&img[lr * EP + ec]);
      if (row >= R) continue;
      if (col + 3 < Cn && (Cn & 3) == 0) {
        *reinterpret_cast<f4*>(out + static_cast<int64_t>(row) * Cn + col) = v;
      } else {
        for (int t2 = 0; t2 < 4 && col + t2 < Cn; ++t2) out[static_cast<int64_t>(row) * Cn + col + t2] = v[t2];
      }
    }
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
  }
  if (csum_a) {
    csa += __shfl_xor(csa, 32);
    const int col = n10 + w * 32 + li;
    if (lh == 0 && col < N1) colsum_slab[static_cast<int64_t>(split) * N1 + col] = csa;
  }
  if (csum_b) {
    // the two 8-row halves of each B column: half 1 hands its sum to half 0 through LDS
    __syncthreads();
    float* red = reinterpret_cast<float*>(smem);
#pragma unroll
    for (int u = 0; u < NJ; ++u) {
      const int job = tid + u * NT;
      if (job < JOBS && job / BN == 1) red[job % BN] = csb[u];
    }
    __syncthreads();
#pragma unroll
    for (int u = 0; u < NJ; ++u) {
      const int job = tid + u * NT, col = n20 + job % BN;
      if (job < JOBS && job / BN == 0 && col < N2)
        colsum_slab[static_cast<int64_t>(split) * N2 + col] = csb[u] + red[job % BN];
    }
  }
}

// out[i] = sum_s slab[s][i] in split order (deterministic); 4 independent chains per thread
__global__ void __launch_bounds__(256) x3_slab_reduce(const float* __restrict__ slab, int splits, int64_t n,
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

struct TnPlan {
  bool swap;   // A <-> B (the wider operand goes to the wave-direct side)
  int nw;      // waves per block (32 C rows each)
  int n1, n2;  // sizes after the swap
  int tiles, splits, rows;
};

TnPlan tn_plan(int M, int N1, int N2) {
  TnPlan p;
  p.swap = N2 > N1;
  p.n1 = p.swap ? N2 : N1;
  p.n2 = p.swap ? N1 : N2;
  // 8 waves (256 C rows share each B chunk, one block per CU) when the rows tile exactly: -4 % at 256 x 256,
  // -9 % at 1024 x 256 (tools/gemm_x3_bench.py, r2ah); else 4 (8 waves lose at 288 rows: 0.60 vs 0.49 ms);
  // 3 (96-row tiles, exact for 288) measured slower: fewer threads share the B staging
  p.nw = p.n1 % 256 == 0 ? 8 : 4;
  if (const int v = m2f::option(m2f::kOptX3TnNw, 0)) p.nw = v == 3 ? 3 : v == 8 ? 8 : 4;
  p.tiles = ((p.n1 + 32 * p.nw - 1) / (32 * p.nw)) * ((p.n2 + 255) / 256);
  // ~512 blocks (2 per CU); 768 when the last row tile is partial (the 288-wide sampling projection:
  // 0.52 vs 0.65 ms at M = 344064; full tiles measured best at 512, tools/gemm_x3_bench.py)
  int target = (p.n1 % (32 * p.nw) ? 768 : 512) / (p.nw >= 8 ? 2 : 1);   // 8 waves: one block per CU
  target = std::max(1, m2f::option(m2f::kOptX3TnBlocks, target));
  int splits = (target + p.tiles - 1) / p.tiles;
  const int max_splits = (M + 8 * kBK - 1) / (8 * kBK);       // >= 8 chunks per block
  if (splits > max_splits) splits = max_splits;
  p.splits = splits < 1 ? 1 : splits;
  const int r = (M + p.splits - 1) / p.splits;
  p.rows = (r + kBK - 1) / kBK * kBK;
  return p;
}

}  // namespace

extern "C" int m2f_gemm_f32x3_nt_workspace(int N, int K, int64_t* workspace_bytes) {
  if (N <= 0 || K <= 0) return m2f::fail(M2F_EINVAL, "m2f_gemm_f32x3_nt_workspace: N %d K %d", N, K);
  if (workspace_bytes) *workspace_bytes = nt_workspace(N, K);
  return m2f::ok();
}

namespace {

int nt_impl(const char* fn, const float* A, int64_t lda, const float* B, int64_t ldb, int b_kn, const float* bias,
            int relu, const float* mask, int64_t ldm, const float* D1, const float* D2, int64_t ldd, uint32_t* bits_out,
            const uint32_t* bits_in, int64_t ldbits, float* C, int64_t ldc, int M, int N, int K, void* workspace,
            int64_t workspace_bytes, void* stream, int dper = 0) {
  if (M < 0 || N <= 0 || K <= 0) return m2f::fail(M2F_EINVAL, "%s: M %d N %d K %d", fn, M, N, K);
  if (dper < 0 || (dper && !D1)) return m2f::fail(M2F_EINVAL, "%s: row period %d needs D1", fn, dper);
  if (!A || !B || !C) return m2f::fail(M2F_EINVAL, "%s: null pointer", fn);
  if (K % 4 || lda % 4 || lda < K || ldb < (b_kn ? N : K) || ldc < N || !m2f::aligned(A, 16))
    return m2f::fail(M2F_EINVAL, "%s: K, lda must be multiples of 4 (lda >= K), A 16-byte aligned", fn);
  if (mask && ldm < N) return m2f::fail(M2F_EINVAL, "%s: ldm %lld < N", fn, static_cast<long long>(ldm));
  if (relu && mask) return m2f::fail(M2F_EINVAL, "%s: relu and mask are exclusive", fn);
  if (D2 && !D1) return m2f::fail(M2F_EINVAL, "%s: D2 without D1", fn);
  if (D1 && (relu || mask)) return m2f::fail(M2F_EINVAL, "%s: addends exclude relu and mask", fn);
  if (D1 && (ldd < N || (ldd & 3) || (ldc & 3) || ((N & 3) != 0) || !m2f::aligned(D1, 16) ||
             (D2 && !m2f::aligned(D2, 16)) || !m2f::aligned(C, 16)))
    return m2f::fail(M2F_EINVAL, "%s: addends need ldd >= N, N/ldd/ldc multiples of 4, 16-byte alignment", fn);
  if (bits_out || bits_in) {
    if ((bits_out && bits_in) || (bits_out && !relu) || (bits_in && relu) || mask || D1)
      return m2f::fail(M2F_EINVAL, "%s: bits_out needs relu, bits_in excludes relu; neither with mask or addends", fn);
    if (N % 32 || ldbits < N / 32 || (ldc & 3) || !m2f::aligned(C, 16))
      return m2f::fail(M2F_EINVAL, "%s: mask bits need N %% 32 == 0, ldbits >= N / 32, ldc %% 4 == 0", fn);
  }
  if (!workspace || workspace_bytes < nt_workspace(N, K) || !m2f::aligned(workspace, 16))
    return m2f::fail(M2F_EINVAL, "%s: workspace %lld < %lld (16-byte aligned)", fn,
                     static_cast<long long>(workspace_bytes), static_cast<long long>(nt_workspace(N, K)));
  if (M == 0) return m2f::ok();
  hipStream_t st = static_cast<hipStream_t>(stream);
  const int NP = static_cast<int>(nt_np(N)), nchunks = (K + kBK - 1) / kBK;
  __bf16* Bs = static_cast<__bf16*>(workspace);
  x3_presplit<<<m2f::ceil_div(static_cast<int64_t>(nchunks) * NP, 256), 256, 0, st>>>(B, ldb, b_kn, N, K, NP, nchunks, Bs);
  if (int rc = m2f::check_launch(fn)) return rc;
  const int epi = (bias ? kBias : 0) | (relu ? kRelu : 0) | (mask ? kMask : 0) | (D1 ? kAdd : 0) |
                  (bits_out ? kBitsOut : 0) | (bits_in ? kBitsIn : 0);
  uint32_t* bits = bits_out ? bits_out : const_cast<uint32_t*>(bits_in);
  if (bits) ldm = ldbits;
  // 96-wide columns for N = 3 * 96 k (the 288-wide sampling projection), else 128-wide columns; 8 waves either
  // way (256 rows share one B chunk: 128-wide 0.285 vs 0.321 ms at K = N = 256, 0.913 vs 0.949 at K = 1024, equal
  // at N = 1024, tools/gemm_x3_bench.py, r2af; 96-wide 0.385 -> 0.365 ms at N = 288, profiles/r05_ah_x3_nt_cfg.txt)
  int cfg = (N % 128 != 0 && N % 96 == 0) ? 4 : 3;
  cfg = m2f::option(m2f::kOptX3NtCfg, cfg);
  switch (cfg) {
    case 0: return launch_nt<128, 4>(epi, A, lda, Bs, NP, bias, mask, ldm, D1, D2, ldd, dper, bits, C, ldc, M, N, K, st);
    case 1: return launch_nt<96, 4>(epi, A, lda, Bs, NP, bias, mask, ldm, D1, D2, ldd, dper, bits, C, ldc, M, N, K, st);
    case 2: return launch_nt<256, 4>(epi, A, lda, Bs, NP, bias, mask, ldm, D1, D2, ldd, dper, bits, C, ldc, M, N, K, st);
    case 3: return launch_nt<128, 8>(epi, A, lda, Bs, NP, bias, mask, ldm, D1, D2, ldd, dper, bits, C, ldc, M, N, K, st);
    case 4: return launch_nt<96, 8>(epi, A, lda, Bs, NP, bias, mask, ldm, D1, D2, ldd, dper, bits, C, ldc, M, N, K, st);
    default: return m2f::fail(M2F_EINVAL, "%s: config %d", fn, cfg);
  }
}

}  // namespace

extern "C" int m2f_gemm_f32x3_nt(const float* A, int64_t lda, const float* B, int64_t ldb, int b_kn, const float* bias,
                                 int relu, const float* mask, int64_t ldm, float* C, int64_t ldc, int M, int N, int K,
                                 void* workspace, int64_t workspace_bytes, void* stream) {
  return nt_impl("m2f_gemm_f32x3_nt", A, lda, B, ldb, b_kn, bias, relu, mask, ldm, nullptr, nullptr, 0, nullptr,
                 nullptr, 0, C, ldc, M, N, K, workspace, workspace_bytes, stream);
}

extern "C" int m2f_gemm_f32x3_nt_add(const float* A, int64_t lda, const float* B, int64_t ldb, int b_kn,
                                     const float* bias, int relu, const float* mask, int64_t ldm, const float* D1,
                                     const float* D2, int64_t ldd, float* C, int64_t ldc, int M, int N, int K,
                                     void* workspace, int64_t workspace_bytes, void* stream) {
  return nt_impl("m2f_gemm_f32x3_nt_add", A, lda, B, ldb, b_kn, bias, relu, mask, ldm, D1, D2, ldd, nullptr, nullptr,
                 0, C, ldc, M, N, K, workspace, workspace_bytes, stream);
}

extern "C" int m2f_gemm_f32x3_nt_rowadd(const float* A, int64_t lda, const float* B, int64_t ldb, int b_kn,
                                        const float* R, int64_t ldr, int period, float* C, int64_t ldc, int M, int N,
                                        int K, void* workspace, int64_t workspace_bytes, void* stream) {
  if (!R || period <= 0) return m2f::fail(M2F_EINVAL, "m2f_gemm_f32x3_nt_rowadd: R and a positive period needed");
  return nt_impl("m2f_gemm_f32x3_nt_rowadd", A, lda, B, ldb, b_kn, nullptr, 0, nullptr, 0, R, nullptr, ldr, nullptr,
                 nullptr, 0, C, ldc, M, N, K, workspace, workspace_bytes, stream, period);
}

extern "C" int m2f_gemm_f32x3_nt_bits(const float* A, int64_t lda, const float* B, int64_t ldb, int b_kn,
                                      const float* bias, int relu, uint32_t* bits_out, const uint32_t* bits_in,
                                      int64_t ldbits, float* C, int64_t ldc, int M, int N, int K, void* workspace,
                                      int64_t workspace_bytes, void* stream) {
  if (!bits_out && !bits_in) return m2f::fail(M2F_EINVAL, "m2f_gemm_f32x3_nt_bits: no mask bits");
  return nt_impl("m2f_gemm_f32x3_nt_bits", A, lda, B, ldb, b_kn, bias, relu, nullptr, 0, nullptr, nullptr, 0,
                 bits_out, bits_in, ldbits, C, ldc, M, N, K, workspace, workspace_bytes, stream);
}

extern "C" int m2f_gemm_f32x3_tn_workspace(int M, int N1, int N2, int64_t* workspace_bytes) {
  if (M < 0 || N1 <= 0 || N2 <= 0) return m2f::fail(M2F_EINVAL, "m2f_gemm_f32x3_tn_workspace: bad sizes");
  const TnPlan p = tn_plan(M, N1, N2);
  if (workspace_bytes) *workspace_bytes = static_cast<int64_t>(p.splits) * (static_cast<int64_t>(N1) * N2 + N1) * 4;
  return m2f::ok();
}

extern "C" int m2f_gemm_f32x3_tn(const float* A, int64_t lda, const float* B, int64_t ldb, float* C, int64_t ldc,
                                 float* colsum, int M, int N1, int N2, void* workspace, int64_t workspace_bytes,
                                 void* stream) {
  const char* fn = "m2f_gemm_f32x3_tn";
  if (M < 0 || N1 <= 0 || N2 <= 0) return m2f::fail(M2F_EINVAL, "%s: M %d N1 %d N2 %d", fn, M, N1, N2);
  if ((M > 0 && (!A || !B)) || !C) return m2f::fail(M2F_EINVAL, "%s: null pointer", fn);
  if (lda < N1 || ldb < N2 || ldc < N2) return m2f::fail(M2F_EINVAL, "%s: leading dimensions too small", fn);
  const TnPlan p = tn_plan(M, N1, N2);
  const int64_t need = static_cast<int64_t>(p.splits) * (static_cast<int64_t>(N1) * N2 + N1) * 4;
  if (!workspace || workspace_bytes < need)
    return m2f::fail(M2F_EINVAL, "%s: workspace %lld < %lld", fn, static_cast<long long>(workspace_bytes),
                     static_cast<long long>(need));
  hipStream_t st = static_cast<hipStream_t>(stream);
  float* slab = static_cast<float*>(workspace);
  float* cslab = slab + static_cast<int64_t>(p.splits) * N1 * N2;
  const float* a = p.swap ? B : A;
  const float* b = p.swap ? A : B;
  const int64_t la = p.swap ? ldb : lda, lb = p.swap ? lda : ldb;
  const unsigned grid = static_cast<unsigned>(p.splits * p.tiles);
  // slab orientation is always [N1][N2] (the caller's): transposed store when swapped
  if (M > 0) {
    float* cs = colsum ? cslab : nullptr;
    const int csum = colsum ? (p.swap ? 2 : 1) : 0;
    const bool mfull = M % kBK == 0;
#define M2F_TN(NWV, MF, CS)                                                                                        \
  x3_tn_kernel<NWV, MF, CS><<<grid, 64 * NWV, 0, st>>>(a, la, b, lb, M, p.n1, p.n2, p.rows, p.swap ? 1 : 0, slab, cs, \
                                                       p.swap ? 1 : 0)
#define M2F_TN_CS(NWV, MF) \
  (csum == 0 ? M2F_TN(NWV, MF, 0) : csum == 1 ? M2F_TN(NWV, MF, 1) : M2F_TN(NWV, MF, 2))
    if (p.nw == 3) {
      if (mfull) M2F_TN_CS(3, true); else M2F_TN_CS(3, false);
    } else if (p.nw == 8) {
      if (mfull) M2F_TN_CS(8, true); else M2F_TN_CS(8, false);
    } else {
      if (mfull) M2F_TN_CS(4, true); else M2F_TN_CS(4, false);
    }
#undef M2F_TN_CS
#undef M2F_TN
    if (int rc = m2f::check_launch(fn)) return rc;
  }
  const int64_t n = static_cast<int64_t>(N1) * N2;
  if (M > 0) {
    x3_slab_reduce<<<m2f::ceil_div(n, 256), 256, 0, st>>>(slab, p.splits, n, C, ldc, N2);
    if (int rc = m2f::check_launch(fn)) return rc;
    if (colsum) {
      x3_slab_reduce<<<m2f::ceil_div(N1, 256), 256, 0, st>>>(cslab, p.splits, N1, colsum, N1, N1);
      return m2f::check_launch(fn);
    }
    return m2f::ok();
  }
  // M == 0: C = 0, colsum = 0
  if (m2f::zero2d_f32_async(C, ldc, N2, N1, st) != hipSuccess) return m2f::fail(M2F_ELAUNCH, "%s: zero fill", fn);
  if (colsum && m2f::zero_async(colsum, static_cast<size_t>(N1) * 4, st) != hipSuccess)
    return m2f::fail(M2F_ELAUNCH, "%s: memset", fn);
  return m2f::ok();
}
