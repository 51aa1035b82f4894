// Mask-embed einsum with the attention-bitmask epilogue for gfx950 (reference
// mask2former/modeling/transformer_decoder/mask2former_transformer_decoder.py:437-452 and the video form
// mask2former_video/.../video_mask2former_transformer_decoder.py:444-461).
//
//   masks[b, q, t, n] = sum_c embed[b, q, c] * feats[b, c, t, n]         ("bqc,bchw->bqhw", "bqc,btchw->bqthw";
//                                                                        the video features as the fold holds them)
//
// in bf16 / fp16 (the autocast dtype) on v_mfma_f32_32x32x16_{bf16,f16} with fp32 accumulation, the result
// rounded once to the dtype (what the library GEMM under autocast returns).  When a target size is given the
// same kernel also emits the next cross-attention's mask from the rounded logits: F.interpolate(bilinear,
// align_corners=False) to the target size, sigmoid in the dtype, < 0.5 (:446-449), one bit per (b, q, key)
// shared by the heads -- for the exact integer ratios the pyramid produces (s = H / h = W / w in {2, 4, 8}),
// where target pixel (y, x) reads source rows s*y + s/2 - 1 and s*y + s/2 and the same two columns, with
// weights 1/2 (upsample_bilinear2d's formula, evaluated literally, contraction off).  m2f_mask_row_fix then
// clears rows whose every key is blocked (:400).
//
// Work split: a workgroup (8 waves) owns one (image, frame), two source rows r, r+1 (paired so that every
// target row's two source rows share a workgroup: pairs start at row (s/2 - 1) & 1) and 128 columns; wave w
// computes source row r + w/4, columns 32*(w%4) .. +31, for all queries (QT tiles of 32 rows).  Per 32-deep
// k stage the features' 32 x 256 slab and the embed's QT*32 x 32 slab are staged in LDS (feature rows padded
// to 576 B so the transposed ds_read_b64_tr_b16 of the B operand is conflict-free, embed rows to 80 B for the
// A operand's 16-byte reads), double-buffered, with the next two stages' global loads in flight in registers
// (32 KB per workgroup, two workgroups per CU at QT <= 4).  The epilogue rounds each 32-query tile into LDS,
// stores the rows coalesced and, on a pair that holds a target row, thresholds the 2x2 averages: aligned
// 16-bit runs of bits are stored directly (the pyramid's 32/64/128-wide targets), other widths OR-ed in.
// HBM-bound: the features are read once and the masks written once.
#include "common.h"

#include <cstdint>

namespace {

using s4 = short __attribute__((ext_vector_type(4)));
using s8 = short __attribute__((ext_vector_type(8)));
using f16v = float __attribute__((ext_vector_type(16)));
using bf8 = __bf16 __attribute__((ext_vector_type(8)));
using h8 = _Float16 __attribute__((ext_vector_type(8)));
using lds_s4 = __attribute__((address_space(3))) s4;

constexpr int kCols = 128;               // columns per workgroup
constexpr int kKC = 32;                  // k per stage
constexpr int kFPitch = 2 * kCols + 32;  // LDS pitch of a feature k-row (elements): 576 B
constexpr int kEPitch = kKC + 8;         // LDS pitch of an embed row (elements): 80 B
constexpr int kThreads = 512;

template <typename T> struct MhElt;
template <> struct MhElt<__bf16> {
  __device__ static f16v mma(s8 a, s8 b, f16v c) {
    return __builtin_amdgcn_mfma_f32_32x32x16_bf16(__builtin_bit_cast(bf8, a), __builtin_bit_cast(bf8, b), c, 0, 0, 0);
  }
  __device__ static float to_f(__bf16 x) { return static_cast<float>(x); }
  __device__ static __bf16 from_f(float x) { return static_cast<__bf16>(x); }
};
template <> struct MhElt<_Float16> {
  __device__ static f16v mma(s8 a, s8 b, f16v c) {
    return __builtin_amdgcn_mfma_f32_32x32x16_f16(__builtin_bit_cast(h8, a), __builtin_bit_cast(h8, b), c, 0, 0, 0);
  }
  __device__ static float to_f(_Float16 x) { return static_cast<float>(x); }
  __device__ static _Float16 from_f(float x) { return static_cast<_Float16>(x); }
};

// Transposed 4x16 read: lane 4q+p of each 16-lane group passes the address of row q, columns 4p..4p+3 of
// its block; lane i receives column i of the 4 rows (row q in element q).
__device__ __forceinline__ s4 tr_read(const void* p) {
  return __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s4*)(reinterpret_cast<uintptr_t>(p)));
}

struct MhArgs {
  const void* embed;    // (B, Q, C)
  const void* feats;    // (B, C, T, H, W)
  void* out;            // (B, Q, T, H, W)
  uint32_t* bits;       // (B, Q, nwords) zeroed by the caller, or null
  int B, Q, C, T, H, W;
  int s;                // resize ratio (0: no bits)
  int h, w, nwords;     // target size, words per (b, q) bit row
  int off;              // first paired row (0 or 1)
  int ngroups, ncol;    // row groups per frame, column chunks per row
  int store16;          // every block's run of bits per row is 16-bit aligned: plain stores
};

// one bit per (q, target x) of this workgroup's target row into the (b, q) bit row
__device__ __forceinline__ void emit_bits(const MhArgs& a, int b, int q, int key, bool valid, bool blocked) {
  const int lane = threadIdx.x & 63;
  const unsigned long long bal = __ballot(valid && blocked);
  if (a.store16) {
    // lanes run over consecutive x of one q in whole 16-bit halves: the first lane of each stores them
    if (valid && (key & 15) == 0) {
      uint16_t* dst = reinterpret_cast<uint16_t*>(a.bits) + static_cast<int64_t>(b * a.Q + q) * a.nwords * 2;
      dst[key >> 4] = static_cast<uint16_t>((bal >> lane) & 0xffffu);
    }
    return;
  }
  // general widths: runs of lanes that share a word are merged by their first lane and OR-ed in
  const long long wkey = valid ? (static_cast<long long>(b * a.Q + q) * a.nwords + (key >> 5)) : -1;
  const long long prev = __shfl_up(wkey, 1);
  const bool lead = valid && (lane == 0 || prev != wkey);
  const unsigned long long leaders = __ballot(lead);
  if (!lead) return;
  const unsigned long long after = lane == 63 ? 0ull : (leaders >> (lane + 1));
  const int run = after ? __builtin_ctzll(after) + 1 : 64 - lane;  // lanes up to the next leader
  // lanes past the last valid one never lead and are not blocked: a run may safely include them
  const unsigned long long mine = (bal >> lane) & (run >= 64 ? ~0ull : ((1ull << run) - 1));
  const uint32_t word = static_cast<uint32_t>(mine << (key & 31));
  if (word) atomicOr(a.bits + wkey, word);
}

template <typename T, int QT>
__global__ void __launch_bounds__(kThreads, 1) mask_heads_kernel(MhArgs a) {
  using E = MhElt<T>;
  constexpr int QP = 32 * QT;
  constexpr int EPIECES = QP * (kKC / 8);                   // 16-byte embed pieces per stage
  constexpr int EP = (EPIECES + kThreads - 1) / kThreads;   // per thread
  __shared__ __attribute__((aligned(16))) T sf[2][kKC * kFPitch];
  __shared__ __attribute__((aligned(16))) T se[2][QP * kEPitch];
  __shared__ __attribute__((aligned(16))) T sout[32][2 * kCols + 8];

  // block -> (image b, frame t, row group, column chunk); column chunk fastest
  int id = blockIdx.x;
  const int cc = id % a.ncol;
  id /= a.ncol;
  const int g = id % a.ngroups;
  id /= a.ngroups;
  const int t = id % a.T, b = id / a.T;
  int r0, nrows;
  if (a.off && g == 0) { r0 = 0; nrows = 1; }
  else {
    r0 = a.off + 2 * (g - a.off);
    nrows = min(2, a.H - r0);
  }
  const int c0 = cc * kCols, cw = min(kCols, a.W - c0);

  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const int li = lane & 31, lh = lane >> 5;
  const int rs_w = w >> 2, ct_w = (w & 3) * 32;
  const int64_t HW = static_cast<int64_t>(a.H) * a.W;
  const int64_t kstride = a.T * HW;  // feature stride between channels
  const T* fimg = static_cast<const T*>(a.feats) + static_cast<int64_t>(b) * a.C * kstride + t * HW;
  const T* emb = static_cast<const T*>(a.embed) + static_cast<int64_t>(b) * a.Q * a.C;

  // staging map.  features: piece p = tid + 512 u -> (k row p >> 5, source row (p >> 4) & 1, 8 columns);
  // embed: piece p = tid + 512 u -> (query p >> 2 clamped to Q - 1, 8 k).  Out-of-range feature pieces are 0.
  const int fk0 = tid >> 5, frs = (tid >> 4) & 1, fcol = (tid & 15) * 8;
  const bool fok = frs < nrows && fcol < cw;
  const T* fptr = fimg + static_cast<int64_t>(fk0) * kstride + static_cast<int64_t>(r0 + (fok ? frs : 0)) * a.W + c0 +
                  (fok ? fcol : 0);
  struct Stage {
    s8 f[2];
    s8 e[EP];
  };
  auto gload = [&](int kc, Stage& st) {
#pragma unroll
    for (int u = 0; u < 2; ++u) {
      st.f[u] = s8{0, 0, 0, 0, 0, 0, 0, 0};
      if (fok) st.f[u] = *reinterpret_cast<const s8*>(fptr + static_cast<int64_t>(kc * kKC + 16 * u) * kstride);
    }
#pragma unroll
    for (int u = 0; u < EP; ++u) {
      const int p = tid + u * kThreads;
      if (EPIECES % kThreads == 0 || p < EPIECES) {
        const int q = min(p >> 2, a.Q - 1);
        st.e[u] = *reinterpret_cast<const s8*>(emb + static_cast<int64_t>(q) * a.C + kc * kKC + (p & 3) * 8);
      }
    }
  };
  auto lstore = [&](int buf, const Stage& st) {
#pragma unroll
    for (int u = 0; u < 2; ++u)
      *reinterpret_cast<s8*>(&sf[buf][(fk0 + 16 * u) * kFPitch + frs * kCols + fcol]) = st.f[u];
#pragma unroll
    for (int u = 0; u < EP; ++u) {
      const int p = tid + u * kThreads;
      if (EPIECES % kThreads == 0 || p < EPIECES)
        *reinterpret_cast<s8*>(&se[buf][(p >> 2) * kEPitch + (p & 3) * 8]) = st.e[u];
    }
  };

  f16v acc[QT];
#pragma unroll
  for (int qt = 0; qt < QT; ++qt)
#pragma unroll
    for (int e = 0; e < 16; ++e) acc[qt][e] = 0.f;

  // B operand: lane (group gq = lane >> 4): k rows 16 h2 + 8 lh + 4 v + qq, columns ct_w + 16 (gq & 1) + 4 pp
  // of the wave's source row (lane 4 qq + pp supplies that address)
  const int gq = lane >> 4, qq = (lane & 15) >> 2, pp = lane & 3;
  const int bcol = rs_w * kCols + ct_w + 16 * (gq & 1) + 4 * pp;
  const int nk = a.C / kKC;
  Stage p1, p2;
  gload(0, p1);
  lstore(0, p1);
  if (nk > 1) gload(1, p1);
  __syncthreads();
  for (int kc = 0; kc < nk; ++kc) {
    const int buf = kc & 1;
    if (kc + 2 < nk) gload(kc + 2, p2);  // stages kc + 1 (p1) and kc + 2 (p2) in flight
    const T* fb = &sf[buf][0];
    const T* eb = &se[buf][0];
#pragma unroll
    for (int h2 = 0; h2 < 2; ++h2) {
      const s4 lo = tr_read(fb + (16 * h2 + 8 * lh + qq) * kFPitch + bcol);
      const s4 hi = tr_read(fb + (16 * h2 + 8 * lh + 4 + qq) * kFPitch + bcol);
      const s8 bfrag = {lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
#pragma unroll
      for (int qt = 0; qt < QT; ++qt) {
        const s8 af = *reinterpret_cast<const s8*>(eb + (32 * qt + li) * kEPitch + 16 * h2 + 8 * lh);
        acc[qt] = E::mma(af, bfrag, acc[qt]);
      }
    }
    if (kc + 1 < nk) lstore(buf ^ 1, p1);
    p1 = p2;
    __syncthreads();
  }

  // ---- epilogue, one q tile at a time: round to T into LDS, coalesced stores, then the bits -----------
  T* out = static_cast<T*>(a.out);
  const bool bits_row = a.s > 0 && nrows == 2 && ((r0 + 1 - (a.s >> 1)) % a.s) == 0;
  const int ty = bits_row ? (r0 + 1 - (a.s >> 1)) / a.s : 0;
#pragma unroll
  for (int qt = 0; qt < QT; ++qt) {
    // C map of 32x32x16: lane column li, rows (e & 3) + 8 (e >> 2) + 4 lh
#pragma unroll
    for (int e = 0; e < 16; ++e) sout[(e & 3) + 8 * (e >> 2) + 4 * lh][rs_w * kCols + ct_w + li] = E::from_f(acc[qt][e]);
    __syncthreads();
    // stores: 32 q x 2 rows x 128 columns in 16-byte pieces, 2 per thread
#pragma unroll
    for (int u = 0; u < 2; ++u) {
      const int piece = tid + u * kThreads;
      const int qr = piece >> 5, rs = (piece >> 4) & 1, col = (piece & 15) * 8;
      const int q = 32 * qt + qr;
      if (q < a.Q && rs < nrows && col < cw) {
        T* dst = out + ((static_cast<int64_t>(b) * a.Q + q) * a.T + t) * HW + static_cast<int64_t>(r0 + rs) * a.W + c0 + col;
        *reinterpret_cast<s8*>(dst) = *reinterpret_cast<const s8*>(&sout[qr][rs * kCols + col]);
      }
    }
    if (bits_row) {
      // target columns of this chunk: x in [c0 / s, (c0 + cw) / s)
#pragma clang fp contract(off)
      const int nx = cw / a.s, x0 = c0 / a.s, hs = (a.s >> 1) - 1;
      const int total = 32 * nx;
      for (int base = w * 64; base < ((total + 63) & ~63); base += kThreads) {
        const int i = base + lane;
        const bool valid = i < total && 32 * qt + i / nx < a.Q;
        const int qr = valid ? i / nx : 0, x = valid ? i - qr * nx : 0;
        bool blocked = false;
        if (valid) {
          const int cl = a.s * x + hs;  // left source column within the chunk
          const float va = E::to_f(sout[qr][cl]), vb = E::to_f(sout[qr][cl + 1]);
          const float vc = E::to_f(sout[qr][kCols + cl]), vd = E::to_f(sout[qr][kCols + cl + 1]);
          const float v = 0.5f * (0.5f * va + 0.5f * vb) + 0.5f * (0.5f * vc + 0.5f * vd);
          const float vt = E::to_f(E::from_f(v));
          const float sg = E::to_f(E::from_f(1.f / (1.f + expf(-vt))));
          blocked = sg < 0.5f;
        }
        const int key = (t * a.h + ty) * a.w + x0 + x;
        emit_bits(a, b, 32 * qt + qr, key, valid, blocked);
      }
    }
    __syncthreads();
  }
}

// fully-masked-row fix (:400): a (b, q) row whose every key is blocked becomes all-unblocked (one wave a row)
__global__ void __launch_bounds__(256) mask_row_fix_kernel(uint32_t* __restrict__ bits, int rows, int nwords,
                                                           int keys) {
  const int row = blockIdx.x * 4 + (threadIdx.x >> 6);
  if (row >= rows) return;  // whole waves
  const int lane = threadIdx.x & 63;
  uint32_t* r = bits + static_cast<int64_t>(row) * nwords;
  const int kw = (keys + 31) / 32;
  const uint32_t tail = (keys & 31) ? ((1u << (keys & 31)) - 1u) : ~0u;
  bool open = false;
  for (int i = lane; i < kw; i += 64) open |= r[i] != (i == kw - 1 ? tail : ~0u);
  if (__ballot(open)) return;
  for (int i = lane; i < nwords; i += 64) r[i] = 0u;
}

// ---- backward --------------------------------------------------------------------------------------------
// d embed = G F^T per head (G = d masks (B, Q, N), F = features (B, C, N), both N-contiguous).  Split over
// N: grid (splits, B); each block computes the whole (Q padded to 32) x 256 partial of its N range into
// part[b][split][q][c] (fp32, q < Q), summed in a fixed order by mask_de_reduce_kernel.  8 waves; wave w:
// channels 64 (w % 4) .. + 63 (two 32-tiles) x query tiles QT (w / 4) .. + QT - 1 (QT = 2 up to 128
// queries, 4 up to 256: config 4's Q = 200, mask2former_transformer_decoder.py:442).  Per 64-deep k step both
// operands are staged in LDS as rows of 64 k (144-B pitch: the 16-byte A and B fragment reads of a 16-lane
// pass cover the 64 banks once): 8 consecutive lanes load one 128-byte row segment, so every global load
// instruction reads whole lines (the former per-wave F fragment loads read 32-byte pieces of 32 rows and ran
// the kernel at 3 TB/s).  One LDS image; the next step's loads are issued right after it is written and land
// during the step's MFMAs.  HBM-bound: G and F are read once.
constexpr int kDeThreads = 512, kDeK = 64, kDePitch = kDeK + 8;

template <typename T, int QT>
__global__ void __launch_bounds__(kDeThreads, QT <= 2 ? 4 : 2) mask_de_kernel(const T* __restrict__ G,
                                                                              const T* __restrict__ F, int Q,
                                                                              int64_t N, int64_t ks, int splits,
                                                                              float* __restrict__ part) {
  using E = MhElt<T>;
  constexpr int C = 256, QP = 64 * QT;                // queries staged (two groups of QT 32-tiles)
  constexpr int GP = QP * (kDeK / 8), FP = C * (kDeK / 8);   // 16-byte pieces per step
  constexpr int GPT = GP / kDeThreads, FPT = FP / kDeThreads;
  __shared__ __attribute__((aligned(16))) T sg[QP * kDePitch];
  __shared__ __attribute__((aligned(16))) T sf[C * kDePitch];
  const int s = blockIdx.x, b = blockIdx.y;
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6, li = lane & 31, lh = lane >> 5;
  const int wc = w & 3, q0 = 32 * QT * (w >> 2);      // channel group, first query of this wave's tiles
  const int64_t k0 = s * ks, k1 = min(N, k0 + ks);
  const int nsteps = static_cast<int>((k1 - k0 + kDeK - 1) / kDeK);
  const T* gb = G + static_cast<int64_t>(b) * Q * N;
  const T* fb = F + static_cast<int64_t>(b) * C * N;
  s8 rg[GPT], rf[FPT];
  // piece p: row p / 8, k 8 (p % 8): 8 consecutive lanes read one row's 128-byte segment.  Past k1 (the
  // last split's tail; k1 is a multiple of 8) or past Q the pieces are zero
  auto load = [&](int step) {
    const int64_t kb = k0 + static_cast<int64_t>(step) * kDeK;
#pragma unroll
    for (int u = 0; u < GPT; ++u) {
      const int p = tid + u * kDeThreads, row = p >> 3, kp = (p & 7) * 8;
      rg[u] = s8{0, 0, 0, 0, 0, 0, 0, 0};
      if (row < Q && kb + kp < k1) rg[u] = *reinterpret_cast<const s8*>(gb + static_cast<int64_t>(row) * N + kb + kp);
    }
#pragma unroll
    for (int u = 0; u < FPT; ++u) {
      const int p = tid + u * kDeThreads, row = p >> 3, kp = (p & 7) * 8;
      rf[u] = s8{0, 0, 0, 0, 0, 0, 0, 0};
      if (kb + kp < k1) rf[u] = *reinterpret_cast<const s8*>(fb + static_cast<int64_t>(row) * N + kb + kp);
    }
  };
  auto store = [&]() {
#pragma unroll
    for (int u = 0; u < GPT; ++u) {
      const int p = tid + u * kDeThreads;
      *reinterpret_cast<s8*>(&sg[(p >> 3) * kDePitch + (p & 7) * 8]) = rg[u];
    }
#pragma unroll
    for (int u = 0; u < FPT; ++u) {
      const int p = tid + u * kDeThreads;
      *reinterpret_cast<s8*>(&sf[(p >> 3) * kDePitch + (p & 7) * 8]) = rf[u];
    }
  };
  f16v acc[QT][2];
#pragma unroll
  for (int qt = 0; qt < QT; ++qt)
#pragma unroll
    for (int j = 0; j < 2; ++j)
#pragma unroll
      for (int e = 0; e < 16; ++e) acc[qt][j][e] = 0.f;
  if (nsteps > 0) load(0);
  for (int t = 0; t < nsteps; ++t) {
    __syncthreads();          // the previous step's fragment reads are done
    store();
    __syncthreads();
    if (t + 1 < nsteps) load(t + 1);
#pragma unroll
    for (int kk = 0; kk < kDeK / 16; ++kk) {
      s8 bf[2];
#pragma unroll
      for (int j = 0; j < 2; ++j)
        bf[j] = *reinterpret_cast<const s8*>(&sf[(64 * wc + 32 * j + li) * kDePitch + 16 * kk + 8 * lh]);
#pragma unroll
      for (int qt = 0; qt < QT; ++qt) {
        const s8 a = *reinterpret_cast<const s8*>(&sg[(q0 + 32 * qt + li) * kDePitch + 16 * kk + 8 * lh]);
#pragma unroll
        for (int j = 0; j < 2; ++j) acc[qt][j] = E::mma(a, bf[j], acc[qt][j]);
      }
    }
  }
  // C map of 32x32x16: lane column li (c), rows (e & 3) + 8 (e >> 2) + 4 lh (q)
  float* out = part + (static_cast<int64_t>(b) * splits + s) * Q * C + 64 * wc + li;
#pragma unroll
  for (int qt = 0; qt < QT; ++qt)
#pragma unroll
    for (int j = 0; j < 2; ++j)
#pragma unroll
      for (int e = 0; e < 16; ++e) {
        const int q = q0 + 32 * qt + (e & 3) + 8 * (e >> 2) + 4 * lh;
        if (q < Q) out[static_cast<int64_t>(q) * C + 32 * j] = acc[qt][j][e];
      }
}

template <typename T>
__global__ void __launch_bounds__(256) mask_de_reduce_kernel(const float* __restrict__ part, int splits,
                                                            int64_t per_b, int64_t total, T* __restrict__ de) {
  const int64_t i = blockIdx.x * static_cast<int64_t>(blockDim.x) + threadIdx.x;
  if (i >= total) return;
  const int64_t b = i / per_b, r = i - b * per_b;
  const float* p = part + b * splits * per_b + r;
  float a0 = 0.f, a1 = 0.f, a2 = 0.f, a3 = 0.f;
  int s = 0;
  for (; s + 3 < splits; s += 4) {
    a0 += p[(s + 0) * per_b];
    a1 += p[(s + 1) * per_b];
    a2 += p[(s + 2) * per_b];
    a3 += p[(s + 3) * per_b];
  }
  for (; s < splits; ++s) a0 += p[s * per_b];
  de[i] = MhElt<T>::from_f((a0 + a1) + (a2 + a3));
}

// d features = sum over heads h of E_h^T G_h, one pass over the heads' G (no concatenation):
// df[b, c, n] = sum_{h, q} Et[b, c, h * QP + q] G_h[b, q, n], Et the embeds transposed and zero-padded to QP
// (a multiple of 16) queries per head, stored in the MFMA A-fragment order (bm2f.h).  Block = (image, 128
// columns of n), 4 waves, wave w: channels 64 w .. 64 w + 63 (two 32-tiles) x the four 32-column tiles.  Per
// k-step (16 queries of one head) the G rows are staged in LDS (rows padded to 320 B: the transposed
// ds_read_b64_tr_b16 of the B operand is conflict-free), double-buffered with the next stage's global loads in
// registers; the A fragments (Et, L2-resident, one contiguous KB per wave load in fragment order) load straight
// from global memory one stage ahead.  fp32 accumulation, one rounding to T.  Config 2: 0.95 ms; with the G
// loads removed (a timing-only build) 0.71 ms, so the G latency left exposed is about a quarter of the time.
constexpr int kDfCols = 128, kDfPitch = kDfCols + 32, kDfMaxHeads = 16;

struct DfHeads {
  const void* g[kDfMaxHeads];
};

// KS: k-steps (16 queries each) per LDS stage.  KS = 4 (the default) stages 64 G rows per barrier: 32 MFMAs per
// wave between barriers instead of 8, the A fragments of a whole stage prefetched one stage ahead.
template <typename T, typename O, int KS = 4>   // O: the features' dtype (T, or fp32 when autocast made T a copy)
__global__ void __launch_bounds__(256, 2) mask_df_kernel(DfHeads heads, const T* __restrict__ Et, int H, int Q,
                                                         int QP, int64_t N, int ncol, O* __restrict__ df) {
  using E = MhElt<T>;
  constexpr int C = 256, KR = 16 * KS;                        // G rows per stage
  constexpr int EPP = 16 / static_cast<int>(sizeof(O));       // output elements per 16-byte piece
  constexpr int GP = KR * kDfCols / 8 / 256;                  // 16-byte G pieces per thread per stage
  __shared__ __attribute__((aligned(16))) T sg[2][KR * kDfPitch];
  __shared__ __attribute__((aligned(16))) O so[4][32][32 + EPP];
  // the heads' G pointers: a per-lane index into the kernel arguments is a global load the G load then waits on
  // (every stage paid two memory round trips); from LDS it is a ds_read
  __shared__ const T* sgp[kDfMaxHeads];
  const int cc = blockIdx.x % ncol, b = blockIdx.x / ncol;
  const int64_t n0 = static_cast<int64_t>(cc) * kDfCols;
  const int cw = static_cast<int>(min<int64_t>(kDfCols, N - n0));
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6, li = lane & 31, lh = lane >> 5;
  const int KP = H * QP, nsteps = KP / 16, nstages = (nsteps + KS - 1) / KS;
  // staging: piece i of a thread -> (stage row (tid >> 4) + 16 i, 8 columns (tid & 15) * 8) of the stage's KR x 128
  // G slab; row k of the K axis is query k % QP of head k / QP (zero past KP and past Q)
  const int scol = (tid & 15) * 8;
  const bool cok = scol < cw;
  const float iqp = 1.f / static_cast<float>(QP);
  auto gload = [&](int stg, s8 (&v)[GP]) {
#pragma unroll
    for (int i = 0; i < GP; ++i) {
      v[i] = s8{0, 0, 0, 0, 0, 0, 0, 0};
      const int k = stg * KR + (tid >> 4) + 16 * i;
      const int h = static_cast<int>((static_cast<float>(k) + 0.5f) * iqp), q = k - h * QP;   // k < 2^16: exact
      if (cok && k < KP && q < Q)
        v[i] = *reinterpret_cast<const s8*>(sgp[h] + (static_cast<int64_t>(b) * Q + q) * N + n0 + scol);
    }
  };
  auto gstore = [&](int buf, const s8 (&v)[GP]) {
#pragma unroll
    for (int i = 0; i < GP; ++i) *reinterpret_cast<s8*>(&sg[buf][((tid >> 4) + 16 * i) * kDfPitch + scol]) = v[i];
  };
  // Et in fragment order: the 16-byte A piece of lane l for (32-channel group, k-step) at
  // ((b * 8 + group) * nsteps + step) * 512 + 8 l -- each A load instruction reads 1 KB contiguous
  const T* et = Et + (static_cast<int64_t>(b) * 8 + 2 * w) * nsteps * 512 + lane * 8;
  f16v acc[2][4];
#pragma unroll
  for (int j = 0; j < 2; ++j)
#pragma unroll
    for (int t = 0; t < 4; ++t)
#pragma unroll
      for (int e = 0; e < 16; ++e) acc[j][t][e] = 0.f;
  const int gq = lane >> 4, qq = (lane & 15) >> 2, pp = lane & 3;
  // A fragments of a stage's KS k-steps (a step past the end clamped to the last: loaded, multiplied by zero rows)
  auto aload = [&](int stg, s8 (&af)[KS][2]) {
#pragma unroll
    for (int s = 0; s < KS; ++s) {
      const int sc = min(stg * KS + s, nsteps - 1);
#pragma unroll
      for (int j = 0; j < 2; ++j) af[s][j] = *reinterpret_cast<const s8*>(et + (static_cast<int64_t>(j) * nsteps + sc) * 512);
    }
  };
  s8 gr[GP], a_cur[KS][2], a_nxt[KS][2];
  if (tid < H) sgp[tid] = static_cast<const T*>(heads.g[tid]);
  __syncthreads();
  gload(0, gr);
  aload(0, a_cur);
  gstore(0, gr);
  __syncthreads();
  for (int stg = 0; stg < nstages; ++stg) {
    const int buf = stg & 1;
    const bool more = stg + 1 < nstages;
    if (more) {  // the next stage's G rows and A fragments in flight during this stage's MFMAs
      gload(stg + 1, gr);
      aload(stg + 1, a_nxt);
    }
    const T* base = &sg[buf][0];
#pragma unroll
    for (int s = 0; s < KS; ++s) {
#pragma unroll
      for (int t = 0; t < 4; ++t) {
        const int col = 32 * t + 16 * (gq & 1) + 4 * pp;
        const s4 lo = tr_read(base + (16 * s + 8 * lh + qq) * kDfPitch + col);
        const s4 hi = tr_read(base + (16 * s + 8 * lh + 4 + qq) * kDfPitch + col);
        const s8 bf = {lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
#pragma unroll
        for (int j = 0; j < 2; ++j) acc[j][t] = E::mma(a_cur[s][j], bf, acc[j][t]);
      }
    }
    if (more) {
      gstore(buf ^ 1, gr);
#pragma unroll
      for (int s = 0; s < KS; ++s) { a_cur[s][0] = a_nxt[s][0]; a_cur[s][1] = a_nxt[s][1]; }
    }
    __syncthreads();
  }
  // epilogue: per 32x32 tile through the wave's LDS image, 16-byte stores (one rounding to O)
  O* out = df + static_cast<int64_t>(b) * C * N + n0;
#pragma unroll
  for (int j = 0; j < 2; ++j)
#pragma unroll
    for (int t = 0; t < 4; ++t) {
#pragma unroll
      for (int e = 0; e < 16; ++e) {
        if constexpr (sizeof(O) == 4) so[w][(e & 3) + 8 * (e >> 2) + 4 * lh][li] = acc[j][t][e];
        else so[w][(e & 3) + 8 * (e >> 2) + 4 * lh][li] = E::from_f(acc[j][t][e]);
      }
      __builtin_amdgcn_wave_barrier();
      __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
#pragma unroll
      for (int u = 0; u < 32 * 32 / EPP / 64; ++u) {
        const int piece = lane + 64 * u, row = piece / (32 / EPP), ce = (piece % (32 / EPP)) * EPP;
        const int col = 32 * t + ce;
        if (col < cw)   // nontemporal: the gradient is not read again here (1-2 % in tools/mask_df_bench.py)
          __builtin_nontemporal_store(*reinterpret_cast<const s8*>(&so[w][row][ce]),
                                      reinterpret_cast<s8*>(out + static_cast<int64_t>(64 * w + 32 * j + row) * N + col));
      }
      __builtin_amdgcn_wave_barrier();
      __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    }
}

template <typename T>
int launch_mask_heads(const MhArgs& a, int QT, hipStream_t st, unsigned grid) {
  switch (QT) {
#define M2F_MH(N) case N: mask_heads_kernel<T, N><<<grid, kThreads, 0, st>>>(a); break;
    M2F_MH(1) M2F_MH(2) M2F_MH(3) M2F_MH(4) M2F_MH(5) M2F_MH(6) M2F_MH(7) M2F_MH(8)
#undef M2F_MH
    default: return m2f::fail(M2F_EUNSUPPORTED, "m2f_mask_heads_fwd: %d queries (at most 256)", 32 * QT);
  }
  return M2F_OK;
}

}  // namespace

extern "C" int m2f_mask_heads_fwd(int dtype, const void* embed, const void* feats, int batch, int num_queries,
                                  int channels, int frames, int height, int width, int target_h, int target_w,
                                  void* masks, uint32_t* bits, int nwords, void* stream) {
  const char* fn = "m2f_mask_heads_fwd";
  if (!embed || !feats || !masks) return m2f::fail(M2F_EINVAL, "%s: null pointer", fn);
  if (dtype != M2F_BF16 && dtype != M2F_F16) return m2f::fail(M2F_EUNSUPPORTED, "%s: dtype %d (bf16 / f16 only)", fn, dtype);
  if (batch <= 0 || num_queries <= 0 || frames <= 0 || height <= 0 || width <= 0)
    return m2f::fail(M2F_EINVAL, "%s: non-positive size", fn);
  if (channels % kKC || channels <= 0 || width % 8)
    return m2f::fail(M2F_EUNSUPPORTED, "%s: channels %% 32 and width %% 8 must be 0 (got %d, %d)", fn, channels, width);
  if (!m2f::aligned(embed, 16) || !m2f::aligned(feats, 16) || !m2f::aligned(masks, 16))
    return m2f::fail(M2F_EINVAL, "%s: 16-byte alignment", fn);
  MhArgs a{};
  a.embed = embed; a.feats = feats; a.out = masks; a.bits = bits;
  a.B = batch; a.Q = num_queries; a.C = channels; a.T = frames; a.H = height; a.W = width;
  a.s = 0; a.off = 0;
  if (target_h > 0) {
    const int s = height / target_h;
    if (s < 2 || (s & 1) || s * target_h != height || s * target_w != width || kCols % s)
      return m2f::fail(M2F_EUNSUPPORTED, "%s: target %dx%d is not an even integer reduction of %dx%d", fn, target_h,
                       target_w, height, width);
    if (!bits) return m2f::fail(M2F_EINVAL, "%s: bits needed with a target", fn);
    if (nwords < (frames * target_h * target_w + 31) / 32) return m2f::fail(M2F_EINVAL, "%s: nwords %d too small", fn, nwords);
    if (!m2f::aligned(bits, 4)) return m2f::fail(M2F_EINVAL, "%s: bits alignment", fn);
    a.s = s; a.h = target_h; a.w = target_w; a.nwords = nwords;
    a.off = ((s >> 1) - 1) & 1;
    // each block's run of a row is 128 / s bits (or the last chunk's (W mod 128) / s) starting at a multiple
    // of the target width: 16-aligned when the target width and every run are multiples of 16
    a.store16 = (target_w % 16 == 0) && (width % (16 * s) == 0) ? 1 : 0;
  }
  a.ngroups = a.off + (height - a.off + 1) / 2;
  a.ncol = (width + kCols - 1) / kCols;
  const int64_t nblocks = static_cast<int64_t>(batch) * frames * a.ngroups * a.ncol;
  if (nblocks > 0x7fffffff) return m2f::fail(M2F_EUNSUPPORTED, "%s: too many workgroups", fn);
  const int QT = (num_queries + 31) / 32;
  hipStream_t st = static_cast<hipStream_t>(stream);
  const int rc = dtype == M2F_BF16 ? launch_mask_heads<__bf16>(a, QT, st, static_cast<unsigned>(nblocks))
                                   : launch_mask_heads<_Float16>(a, QT, st, static_cast<unsigned>(nblocks));
  if (rc) return rc;
  return m2f::check_launch(fn);
}

extern "C" int m2f_mask_row_fix(uint32_t* bits, int rows, int nwords, int keys, void* stream) {
  if (!bits || rows <= 0 || nwords <= 0 || keys <= 0 || (keys + 31) / 32 > nwords)
    return m2f::fail(M2F_EINVAL, "m2f_mask_row_fix: bad arguments");
  mask_row_fix_kernel<<<(rows + 3) / 4, 256, 0, static_cast<hipStream_t>(stream)>>>(bits, rows, nwords, keys);
  return m2f::check_launch("m2f_mask_row_fix");
}

namespace {
int64_t de_splits(int64_t N) {
  // ~512 blocks at bs16 (two per CU), k ranges of whole 64-steps
  const int64_t target = 32;
  int64_t ks = (N + target - 1) / target;
  ks = (ks + kDeK - 1) / kDeK * kDeK;
  return ks < kDeK ? kDeK : ks;
}

template <typename T>
int launch_de(const void* G, const void* F, int B, int Q, int64_t N, float* part, void* de, hipStream_t st) {
  const int64_t ks = de_splits(N);
  const int splits = static_cast<int>((N + ks - 1) / ks);
  const dim3 grid(splits, B);
  const T* g = static_cast<const T*>(G);
  const T* f = static_cast<const T*>(F);
  // two groups of 4 waves split the query tiles: QT = 1 (<= 64 queries), 2 (<= 128), 4 (<= 256)
  if (Q <= 64)
    mask_de_kernel<T, 1><<<grid, kDeThreads, 0, st>>>(g, f, Q, N, ks, splits, part);
  else if (Q <= 128)
    mask_de_kernel<T, 2><<<grid, kDeThreads, 0, st>>>(g, f, Q, N, ks, splits, part);
  else if (Q <= 256)
    mask_de_kernel<T, 4><<<grid, kDeThreads, 0, st>>>(g, f, Q, N, ks, splits, part);
  else
    return m2f::fail(M2F_EUNSUPPORTED, "m2f_mask_heads_bwd_embed: %d queries (at most 256)", Q);
  const int64_t per_b = static_cast<int64_t>(Q) * 256, total = per_b * B;
  mask_de_reduce_kernel<T><<<m2f::ceil_div(total, 256), 256, 0, st>>>(part, splits, per_b, total, static_cast<T*>(de));
  return M2F_OK;
}
}  // namespace

extern "C" int m2f_mask_heads_bwd_workspace(int batch, int num_queries, int64_t n, int64_t* workspace_bytes) {
  if (batch <= 0 || num_queries <= 0 || n <= 0 || !workspace_bytes)
    return m2f::fail(M2F_EINVAL, "m2f_mask_heads_bwd_workspace: bad arguments");
  const int64_t ks = de_splits(n), splits = (n + ks - 1) / ks;
  *workspace_bytes = splits * batch * static_cast<int64_t>(num_queries) * 256 * 4;
  return m2f::ok();
}

extern "C" int m2f_mask_heads_bwd_embed(int dtype, const void* grad_masks, const void* feats, int batch,
                                        int num_queries, int channels, int64_t n, void* grad_embed, void* workspace,
                                        int64_t workspace_bytes, void* stream) {
  const char* fn = "m2f_mask_heads_bwd_embed";
  if (!grad_masks || !feats || !grad_embed || !workspace) return m2f::fail(M2F_EINVAL, "%s: null pointer", fn);
  if (dtype != M2F_BF16 && dtype != M2F_F16) return m2f::fail(M2F_EUNSUPPORTED, "%s: dtype %d", fn, dtype);
  if (channels != 256 || n % 16 || num_queries <= 0 || num_queries > 256 || batch <= 0)
    return m2f::fail(M2F_EUNSUPPORTED, "%s: needs 256 channels, n %% 16 == 0, 1..256 queries", fn);
  if (!m2f::aligned(grad_masks, 16) || !m2f::aligned(feats, 16)) return m2f::fail(M2F_EINVAL, "%s: alignment", fn);
  int64_t need = 0;
  m2f_mask_heads_bwd_workspace(batch, num_queries, n, &need);
  if (workspace_bytes < need) return m2f::fail(M2F_EINVAL, "%s: workspace %lld < %lld", fn,
                                               static_cast<long long>(workspace_bytes), static_cast<long long>(need));
  hipStream_t st = static_cast<hipStream_t>(stream);
  float* part = static_cast<float*>(workspace);
  const int rc = dtype == M2F_BF16 ? launch_de<__bf16>(grad_masks, feats, batch, num_queries, n, part, grad_embed, st)
                                   : launch_de<_Float16>(grad_masks, feats, batch, num_queries, n, part, grad_embed, st);
  if (rc) return rc;
  return m2f::check_launch(fn);
}

extern "C" int m2f_mask_heads_bwd_feats(int dtype, const void* const* grad_masks, int heads, const void* embed_t,
                                        int batch, int num_queries, int padded_queries, int channels, int64_t n,
                                        int out_dtype, void* grad_feats, void* stream) {
  const char* fn = "m2f_mask_heads_bwd_feats";
  if (!grad_masks || !embed_t || !grad_feats) return m2f::fail(M2F_EINVAL, "%s: null pointer", fn);
  if (dtype != M2F_BF16 && dtype != M2F_F16) return m2f::fail(M2F_EUNSUPPORTED, "%s: dtype %d", fn, dtype);
  if (heads <= 0 || heads > kDfMaxHeads || channels != 256 || n % 8 || padded_queries % 16 ||
      padded_queries < num_queries || num_queries <= 0 || batch <= 0)
    return m2f::fail(M2F_EUNSUPPORTED, "%s: needs 1..%d heads, 256 channels, n %% 8 == 0, padded queries %% 16", fn,
                     kDfMaxHeads);
  DfHeads h{};
  for (int i = 0; i < heads; ++i) {
    if (!grad_masks[i] || !m2f::aligned(grad_masks[i], 16)) return m2f::fail(M2F_EINVAL, "%s: head %d pointer", fn, i);
    h.g[i] = grad_masks[i];
  }
  if (!m2f::aligned(embed_t, 16) || !m2f::aligned(grad_feats, 16)) return m2f::fail(M2F_EINVAL, "%s: alignment", fn);
  const int ncol = static_cast<int>((n + kDfCols - 1) / kDfCols);
  const int64_t nblk = static_cast<int64_t>(ncol) * batch;
  if (nblk > 0x7fffffff) return m2f::fail(M2F_EUNSUPPORTED, "%s: too many workgroups", fn);
  hipStream_t st = static_cast<hipStream_t>(stream);
  if (out_dtype != dtype && out_dtype != M2F_F32) return m2f::fail(M2F_EUNSUPPORTED, "%s: out dtype %d", fn, out_dtype);
  const unsigned g = static_cast<unsigned>(nblk);
  const bool ks4 = m2f::option(m2f::kOptMaskDfStage, 4) >= 4;  // k-steps per LDS stage: 4 (default) or 1
#define M2F_DF(T, O)                                                                                                    \
  (ks4 ? mask_df_kernel<T, O, 4><<<g, 256, 0, st>>>(h, static_cast<const T*>(embed_t), heads, num_queries,             \
                                                    padded_queries, n, ncol, static_cast<O*>(grad_feats))              \
       : mask_df_kernel<T, O, 1><<<g, 256, 0, st>>>(h, static_cast<const T*>(embed_t), heads, num_queries,             \
                                                    padded_queries, n, ncol, static_cast<O*>(grad_feats)))
  if (dtype == M2F_BF16) {
    if (out_dtype == M2F_F32) M2F_DF(__bf16, float); else M2F_DF(__bf16, __bf16);
  } else {
    if (out_dtype == M2F_F32) M2F_DF(_Float16, float); else M2F_DF(_Float16, _Float16);
  }
#undef M2F_DF
  return m2f::check_launch(fn);
}
