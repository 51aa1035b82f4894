// Masked-attention decoder kernels for gfx950 (reference
// mask2former/modeling/transformer_decoder/mask2former_transformer_decoder.py).
//
// 1. attn-mask bitmask: forward_prediction_heads' bilinear resize of the mask logits (:446), the
//    `sigmoid() < 0.5` threshold in the logits' dtype (:449) and the next layer's fully-masked-row
//    fix (:400), fused into one pass that writes ONE bit per (b, q, key) shared by all heads instead
//    of the reference's head-repeated (B*h, Q, HW) bool tensor.
// 2. masked cross-attention core: softmax(scale * q k^T  +  mask) v per (b, head), flash style
//    (online softmax, no score matrix in HBM), on 16x16 MFMA tiles (bf16 / fp16: 16x16x16, fp32:
//    16x16x4), key range split over workgroups with a combine pass; backward recomputes P from the
//    saved log-sum-exp.  Replaces the math path of nn.MultiheadAttention(attn_mask=bool) used by
//    CrossAttentionLayer.forward_post (:98-110); the q/k/v/out projections stay dense GEMMs.
//
// MFMA operand maps used throughout (16x16xK, lane = 16*g + r):
//   A: lane holds A[row r][k = kw*g + j]   B: lane holds B[k = kw*g + j][col r]   (kw = 4 for 16-bit, 1 for f32)
//   C: lane holds C[row 4*g + i][col r], i = 0..3
#include "common.h"

#include <cmath>
#include <cstdlib>

namespace {

using f4 = float __attribute__((ext_vector_type(4)));
using s4 = short __attribute__((ext_vector_type(4)));
using h4 = _Float16 __attribute__((ext_vector_type(4)));
using lds_s4 = __attribute__((address_space(3))) s4;

constexpr int kD = 32;       // head dim (hidden 256 / 8 heads)
constexpr float kLazyLog2 = 8.f;   // forward: rescale when a block max exceeds the running max by 2^8
constexpr int kDQ = kD + 1;   // row pitch of the register-dQ reductions' LDS image (floats): at most 2-way bank
                              // conflicts (a pitch of kD puts the 16 lanes of a column group on one bank)
constexpr int kDP = kD + 4;  // padded LDS row (elements) for 16-bit images: 72 B rows, 8 B aligned
constexpr float kLog2e = 1.4426950408889634f;

// ----------------------------------------------------------------------------------------------
// element traits
// ----------------------------------------------------------------------------------------------
template <typename T> struct Elt;
template <> struct Elt<float> {
  static constexpr bool k16 = false;
  __device__ static float to_f(float x) { return x; }
  __device__ static float from_f(float x) { return x; }
};
template <> struct Elt<__bf16> {
  static constexpr bool k16 = true;
  __device__ static float to_f(__bf16 x) { return static_cast<float>(x); }
  __device__ static __bf16 from_f(float x) { return static_cast<__bf16>(x); }
};
template <> struct Elt<_Float16> {
  static constexpr bool k16 = true;
  __device__ static float to_f(_Float16 x) { return static_cast<float>(x); }
  __device__ static _Float16 from_f(float x) { return static_cast<_Float16>(x); }
};

template <typename T>
__device__ __forceinline__ f4 mma16(s4 a, s4 b, f4 c) {
  if constexpr (std::is_same<T, _Float16>::value)
    return __builtin_amdgcn_mfma_f32_16x16x16f16(__builtin_bit_cast(h4, a), __builtin_bit_cast(h4, b), c, 0, 0, 0);
  else
    return __builtin_amdgcn_mfma_f32_16x16x16bf16_1k(a, b, c, 0, 0, 0);
}

__device__ __forceinline__ f4 mma32(float a, float b, f4 c) {
  return __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, c, 0, 0, 0);
}

// gfx950's 16x16x32 forms (twice the K of 16x16x16 per instruction): lane 16g + r holds A[row r][k = 8g + j] and
// B[k = 8g + j][col r], j = 0..7
using s8 = short __attribute__((ext_vector_type(8)));
using h8 = _Float16 __attribute__((ext_vector_type(8)));
using b8 = __bf16 __attribute__((ext_vector_type(8)));
template <typename T>
__device__ __forceinline__ f4 mmak32(s8 a, s8 b, f4 c) {
  if constexpr (std::is_same<T, _Float16>::value)
    return __builtin_amdgcn_mfma_f32_16x16x32_f16(__builtin_bit_cast(h8, a), __builtin_bit_cast(h8, b), c, 0, 0, 0);
  else
    return __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(b8, a), __builtin_bit_cast(b8, b), c, 0, 0, 0);
}
__device__ __forceinline__ s8 cat8(s4 lo, s4 hi) { return __builtin_shufflevector(lo, hi, 0, 1, 2, 3, 4, 5, 6, 7); }

// x with bit POS of `word` set replaced by -inf: v_bfe_i32 makes the bit a 0 / all-ones mask and v_bfi_b32 selects
// (two VALU; a bit test is and + compare + select).  Builtins, not inline asm: the hazard recognizer must see these
// VALU writes (an MFMA reading a VGPR that the previous instruction wrote needs wait states)
template <int POS>
__device__ __forceinline__ float mask_ninf(uint32_t word, float x) {
  const uint32_t m = static_cast<uint32_t>(__builtin_amdgcn_sbfe(static_cast<int>(word), POS, 1));
  return __uint_as_float((m & 0xff800000u) | (~m & __float_as_uint(x)));
}
// x where bit `pos` of `kept` (an inverted mask word: bit set = key visible) is set, else 0 (v_bfe + v_and)
__device__ __forceinline__ float keep_bit(uint32_t kept, uint32_t pos, float x) {
  const uint32_t m = static_cast<uint32_t>(__builtin_amdgcn_sbfe(static_cast<int>(kept), pos, 1));
  return __uint_as_float(m & __float_as_uint(x));
}
// raw v_exp_f32 (2^x; -inf -> 0): the scores' exponents are <= 0, where exp2f's denormal range reduction only
// changes results below 2^-126
__device__ __forceinline__ float ex2(float x) { return __builtin_amdgcn_exp2f(x); }

template <typename T>
__device__ __forceinline__ s4 pack4(float a, float b, float c, float d) {
  T t[4] = {Elt<T>::from_f(a), Elt<T>::from_f(b), Elt<T>::from_f(c), Elt<T>::from_f(d)};
  return *reinterpret_cast<s4*>(t);
}

// Transposed 4x16 read: lane 4q+p of each 16-lane group passes the address of row q, columns
// 4p..4p+3 of its block; lane i receives column i of the 4 rows (row q in element q).
__device__ __forceinline__ s4 tr_read(const void* lds_ptr) {
  return __builtin_amdgcn_ds_read_tr16_b64_v4i16(
      (lds_s4*)(reinterpret_cast<uintptr_t>(lds_ptr)));
}

// Reduce over the 4 lane groups (same r) with gfx950's row-swap moves (VALU; __shfl_xor is an LDS permute with
// its round trip): v_permlane16_swap pairs rows 0-1 and 2-3 (lane ^ 16), v_permlane32_swap the halves (lane ^ 32).
// With both operands the same value, the swapped pair holds {x_lo, x_hi} in every lane of the pair: the sum is
// x_lo + x_hi on both sides (the order __shfl_xor's x + x^16 gives, float addition being commutative).
__device__ __forceinline__ float xor16_pair(float x, float& other) {
  const auto p = __builtin_amdgcn_permlane16_swap(__float_as_uint(x), __float_as_uint(x), false, false);
  other = __uint_as_float(p[1]);
  return __uint_as_float(p[0]);
}
__device__ __forceinline__ float xor32_pair(float x, float& other) {
  const auto p = __builtin_amdgcn_permlane32_swap(__float_as_uint(x), __float_as_uint(x), false, false);
  other = __uint_as_float(p[1]);
  return __uint_as_float(p[0]);
}
__device__ __forceinline__ float wave_max16(float x) {
  float b;
  float a = xor16_pair(x, b);
  x = fmaxf(a, b);
  a = xor32_pair(x, b);
  return fmaxf(a, b);
}
__device__ __forceinline__ float wave_sum16(float x) {
  float b;
  float a = xor16_pair(x, b);
  x = a + b;
  a = xor32_pair(x, b);
  return a + b;
}

// ----------------------------------------------------------------------------------------------
// 1. attention-mask bits
// ----------------------------------------------------------------------------------------------
// One workgroup per (b, q) row.  value at target pixel (y, x) follows upsample_bilinear2d
// (align_corners=False): src = max(scale*(dst+0.5)-0.5, 0), i0 = (int)src, i1 = i0 + (i0 < in-1),
// lambda = src - i0; accumulated in fp32 and rounded to T; then s = T(1/(1+exp(-v))) and
// blocked = s < 0.5.  Contraction is disabled so the arithmetic is the literal formula.
template <typename T>
__global__ void __launch_bounds__(256) attn_mask_bits_kernel(const T* __restrict__ logits, int frames, int Hin,
                                                             int Win, int Hout, int Wout, int nwords, int row_fix,
                                                             uint32_t* __restrict__ bits) {
#pragma clang fp contract(off)
  extern __shared__ uint32_t sbits[];
  __shared__ int sblocked;
  const int64_t row = blockIdx.x;
  const int64_t frame_elems = static_cast<int64_t>(Hin) * Win;
  const T* src_row = logits + row * frames * frame_elems;
  const int HWo = Hout * Wout;
  const int HW = frames * HWo;  // keys of the row: frame-major, then row-major pixels
  const float rh = static_cast<float>(Hin) / static_cast<float>(Hout);
  const float rw = static_cast<float>(Win) / static_cast<float>(Wout);
  if (threadIdx.x == 0) sblocked = 0;
  __syncthreads();
  int count = 0;
  for (int base = 0; base < nwords * 32; base += 256) {
    const int pix = base + threadIdx.x;
    bool blocked = false;
    if (pix < HW) {
      const int f = pix / HWo, fp = pix - f * HWo;
      const T* src = src_row + f * frame_elems;
      const int y = fp / Wout, x = fp - y * Wout;
      float sy = rh * (static_cast<float>(y) + 0.5f) - 0.5f;
      sy = sy < 0.f ? 0.f : sy;
      float sx = rw * (static_cast<float>(x) + 0.5f) - 0.5f;
      sx = sx < 0.f ? 0.f : sx;
      const int y0 = static_cast<int>(sy), x0 = static_cast<int>(sx);
      const int yp = (y0 < Hin - 1) ? 1 : 0, xp = (x0 < Win - 1) ? 1 : 0;
      const float ly1 = sy - static_cast<float>(y0), ly0 = 1.f - ly1;
      const float lx1 = sx - static_cast<float>(x0), lx0 = 1.f - lx1;
      const float a = Elt<T>::to_f(src[y0 * Win + x0]);
      const float b = Elt<T>::to_f(src[y0 * Win + x0 + xp]);
      const float c = Elt<T>::to_f(src[(y0 + yp) * Win + x0]);
      const float d = Elt<T>::to_f(src[(y0 + yp) * Win + x0 + xp]);
      const float v = ly0 * (lx0 * a + lx1 * b) + ly1 * (lx0 * c + lx1 * d);
      const float vt = Elt<T>::to_f(Elt<T>::from_f(v));
      const float s = Elt<T>::to_f(Elt<T>::from_f(1.f / (1.f + expf(-vt))));
      blocked = s < 0.5f;
    }
    const unsigned long long bal = __ballot(blocked);
    count += blocked ? 1 : 0;
    const int lane = threadIdx.x & 63;
    const int word = (base + (threadIdx.x & ~63)) >> 5;
    if (lane == 0 && word < nwords) sbits[word] = static_cast<uint32_t>(bal);
    if (lane == 32 && word + 1 < nwords) sbits[word + 1] = static_cast<uint32_t>(bal >> 32);
  }
  // row total
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) count += __shfl_xor(count, o);
  if ((threadIdx.x & 63) == 0) atomicAdd(&sblocked, count);
  __syncthreads();
  const bool all_blocked = row_fix && sblocked == HW;
  uint32_t* dst = bits + row * nwords;
  for (int w = threadIdx.x; w < nwords; w += 256) dst[w] = all_blocked ? 0u : sbits[w];
}

// ----------------------------------------------------------------------------------------------
// 2. masked attention forward
// ----------------------------------------------------------------------------------------------
// grid (B*H, nchunks), 256 threads.  Wave w owns query tiles w, w+4, ... (TPW of them).  Keys are
// streamed in blocks of 64 through a double-buffered LDS image; S^T = K Q^T is computed so that the
// query is the lane's MFMA column: the online-softmax row statistics are in-lane plus two shuffles,
// and P^T is already the B operand of O^T += V^T P^T.
template <typename T>
struct KVImage {
  static constexpr int RS = Elt<T>::k16 ? kDP : (kD + 1);  // row stride (elements)
  static constexpr int ELEMS = 64 * RS;
};

// CLAMP: rows past the chunk repeat its last row (loads without exec branches, so the compiler's wait counting does
// not stall the prefetch; the forward masks those keys: p = 0 on a row of the input); else they are zero
template <typename T, bool CLAMP = false>
__device__ __forceinline__ void stage_load(const T* __restrict__ src, int64_t row0, int nrows_valid, int stride,
                                           int col0, f4 (&reg)[2]) {
  // 64 rows x 32 elements; 16-bit: 256 x 16 B (one per thread); f32: 512 x 16 B (two per thread)
  constexpr int PER = Elt<T>::k16 ? 8 : 4;
  constexpr int PARTS = kD / PER;
  constexpr int ITERS = Elt<T>::k16 ? 1 : 2;
#pragma unroll
  for (int it = 0; it < ITERS; ++it) {
    const int idx = threadIdx.x + it * 256;
    const int rr = idx / PARTS, part = idx % PARTS;
    if constexpr (CLAMP) {
      reg[it] = *reinterpret_cast<const f4*>(src + (row0 + min(rr, nrows_valid - 1)) * stride + col0 + part * PER);
    } else {
      if (rr < nrows_valid)
        reg[it] = *reinterpret_cast<const f4*>(src + (row0 + rr) * stride + col0 + part * PER);
      else
        reg[it] = f4{0.f, 0.f, 0.f, 0.f};
    }
  }
}

template <typename T>
__device__ __forceinline__ void stage_store(T* img, const f4 (&reg)[2]) {
  constexpr int PER = Elt<T>::k16 ? 8 : 4;
  constexpr int PARTS = kD / PER;
  constexpr int ITERS = Elt<T>::k16 ? 1 : 2;
  constexpr int RS = KVImage<T>::RS;
#pragma unroll
  for (int it = 0; it < ITERS; ++it) {
    const int idx = threadIdx.x + it * 256;
    const int rr = idx / PARTS, part = idx % PARTS;
    T* dst = img + rr * RS + part * PER;
    if constexpr (Elt<T>::k16) {
      // 72 B rows: 8 B aligned, store as two 8 B halves
      const s4* s = reinterpret_cast<const s4*>(&reg[it]);
      reinterpret_cast<s4*>(dst)[0] = s[0];
      reinterpret_cast<s4*>(dst)[1] = s[1];
    } else {
      const float* s = reinterpret_cast<const float*>(&reg[it]);
#pragma unroll
      for (int e = 0; e < 4; ++e) dst[e] = s[e];
    }
  }
}

// the four masks of one 16-key tile's C fragment (keys 4g + i of the tile, bits B0 + i of the lane's pre-shifted word)
template <int B0>
__device__ __forceinline__ void mask4(f4& s, uint32_t word) {
  s[0] = mask_ninf<B0>(word, s[0]);
  s[1] = mask_ninf<B0 + 1>(word, s[1]);
  s[2] = mask_ninf<B0 + 2>(word, s[2]);
  s[3] = mask_ninf<B0 + 3>(word, s[3]);
}

// Per score element: two VALU for the mask (blocked keys and keys past the chunk are both bits of the lane's mask
// words, folded in when the words are loaded), a max3 share, one fma and v_exp for p = 2^(s sl2 - m), half a pack;
// the row sums come from the MFMA (16-bit: an all-ones A operand against P^T).  16-bit operands run on the 16x16x32
// form: S^T tile = one MFMA per 16 keys (K = head dim 32), O^T += V^T P^T one per 32 keys, the key order inside the
// K = 32 step permuted so that P's C fragments of two key tiles are the B operand as they are (element j < 4: key
// 4g + j of the first tile, j >= 4: of the second) and V^T's A operand is two transposed reads of those tiles.
// Workgroup -> (b * H + h, key chunk c) of a (B * H, nchunks) grid.  xmap = 1: the H heads of one (image, chunk) on
// one XCD, one after another (workgroups are dealt to the 8 XCDs round-robin by linear id).  A head's K / V slice is
// 64 bytes of each 512-byte key row (16-bit, 8 heads); with the plain mapping head h runs on XCD h (H = 8), so every
// XCD's L2 fetched whole 128-byte lines for half of them (FETCH_SIZE 2.2-2.3x the K / V bytes).  The host sets xmap
// only when B * nchunks % 8 == 0 (then L = 8t + x, h = t % H, b * nchunks + c = (t / H) * 8 + x is a bijection).
__device__ __forceinline__ void mattn_block(int H, int xmap, int& bh, int& c) {
  if (xmap) {
    const int L = blockIdx.x + gridDim.x * blockIdx.y;
    const int x = L & 7, t = L >> 3;
    const int grp = (t / H) * 8 + x;
    c = grp % gridDim.y;
    bh = (grp / gridDim.y) * H + t % H;
  } else {
    bh = blockIdx.x;
    c = blockIdx.y;
  }
}

template <typename T, int TPW>
__global__ void __launch_bounds__(256, TPW <= 2 ? 4 : TPW <= 4 ? 2 : 1) mattn_fwd_kernel(
    const T* __restrict__ q, const T* __restrict__ k, const T* __restrict__ v, const uint32_t* __restrict__ bits,
    int Lq, int Lk, int H, int qs, int kvs, int nw, float sl2, int chunk_len, T* __restrict__ out,
    float* __restrict__ lse2, float* __restrict__ ws_o, float* __restrict__ ws_ml, int xmap) {
  constexpr bool k16 = Elt<T>::k16;
  constexpr int RS = KVImage<T>::RS;
  __shared__ T Ks[2][KVImage<T>::ELEMS];
  __shared__ T Vs[2][KVImage<T>::ELEMS];
  int bh, c;
  mattn_block(H, xmap, bh, c);
  const int b = bh / H, h = bh % H;
  const int nchunks = gridDim.y;
  const int key_begin = c * chunk_len;
  const int key_end = min(Lk, key_begin + chunk_len);
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6, g = lane >> 4, r = lane & 15;
  const int64_t kvrow0 = static_cast<int64_t>(b) * Lk;

  // query operands (B of S^T = K Q^T): 16-bit: lane holds Q[q = tile*16 + r][d = 8g + j]; f32: [d = dc*4 + g]
  s8 qb16[TPW];
  float qb32[TPW][8];
  f4 o[TPW][2];
  f4 lsum[TPW];  // 16-bit: P's row sums (every element: query r's)
  float m_run[TPW], l_run[TPW];
  uint32_t mrow_ok[TPW];
  // 1.0 in the operand format (f16 0x3C00, bf16 0x3F80)
  constexpr short kOne = std::is_same<T, _Float16>::value ? short(0x3C00) : short(0x3F80);
  const s8 ones = {kOne, kOne, kOne, kOne, kOne, kOne, kOne, kOne};
#pragma unroll
  for (int t = 0; t < TPW; ++t) {
    const int qi = (w + 4 * t) * 16 + r;
    const bool ok = qi < Lq;
    mrow_ok[t] = ok;
    const T* qrow = q + (static_cast<int64_t>(b) * Lq + (ok ? qi : 0)) * qs + h * kD;
    if constexpr (k16) {
      const s4 lo = *reinterpret_cast<const s4*>(qrow + 8 * g);
      const s4 hi = *reinterpret_cast<const s4*>(qrow + 8 * g + 4);
      qb16[t] = ok ? cat8(lo, hi) : s8{0, 0, 0, 0, 0, 0, 0, 0};
    } else {
#pragma unroll
      for (int dc = 0; dc < 8; ++dc) qb32[t][dc] = ok ? Elt<T>::to_f(qrow[dc * 4 + g]) : 0.f;
    }
    o[t][0] = f4{0.f, 0.f, 0.f, 0.f};
    o[t][1] = f4{0.f, 0.f, 0.f, 0.f};
    lsum[t] = f4{0.f, 0.f, 0.f, 0.f};
    m_run[t] = -INFINITY;
    l_run[t] = 0.f;
  }

  f4 kreg[2], vreg[2];
  // this lane's mask words of a 64-key block (query row qi of tile t), loaded one block ahead with K / V
  uint32_t mw[TPW][2];
  // (unconditional loads at clamped addresses: a query row past Lq and a word past the row are overridden when the
  // words are used)
  auto mload = [&](int kb) {
    const int w1 = min((kb >> 5) + 1, nw - 1);
#pragma unroll
    for (int t = 0; t < TPW; ++t) {
      const uint32_t* mr = bits + (static_cast<int64_t>(b) * Lq + min((w + 4 * t) * 16 + r, Lq - 1)) * nw;
      mw[t][0] = mr[kb >> 5];
      mw[t][1] = mr[w1];
    }
  };
  uint32_t mcur[TPW][2];
  int buf = 0;
  if (key_begin < key_end) {
    stage_load<T, true>(k, kvrow0 + key_begin, key_end - key_begin, kvs, h * kD, kreg);
    stage_load<T, true>(v, kvrow0 + key_begin, key_end - key_begin, kvs, h * kD, vreg);
    mload(key_begin);
    stage_store<T>(Ks[0], kreg);
    stage_store<T>(Vs[0], vreg);
  }
  __syncthreads();

  for (int kb0 = key_begin; kb0 < key_end; kb0 += 64) {
    const int next = kb0 + 64;
    {
      // keys past the chunk set as blocked, then the words shifted by 4g: key 16 kt + 4g + i of the block is bit
      // 16 (kt & 1) + i of word kt >> 1 (done here, not at the load, so nothing waits on the prefetch below)
      const int kv = key_end - kb0;  // >= 1
      const uint32_t x0 = kv >= 32 ? 0u : (0xffffffffu << (kv & 31));
      const uint32_t x1 = kv >= 64 ? 0u : (kv <= 32 ? 0xffffffffu : (0xffffffffu << ((kv - 32) & 31)));
      const uint32_t xw = (kb0 >> 5) + 1 < nw ? 0u : 0xffffffffu;  // no second word: keys past Lk
#pragma unroll
      for (int t = 0; t < TPW; ++t) {
        const uint32_t xr = mrow_ok[t] ? 0u : 0xffffffffu;
        mcur[t][0] = (mw[t][0] | x0 | xr) >> (4 * g);
        mcur[t][1] = (mw[t][1] | x1 | xw | xr) >> (4 * g);
      }
    }
    if (next < key_end) {  // prefetch the next block into registers
      stage_load<T, true>(k, kvrow0 + next, key_end - next, kvs, h * kD, kreg);
      stage_load<T, true>(v, kvrow0 + next, key_end - next, kvs, h * kD, vreg);
      mload(next);
    }
    const T* Kc = Ks[buf];
    const T* Vc = Vs[buf];
#pragma unroll
    for (int t = 0; t < TPW; ++t) {
      if ((w + 4 * t) * 16 >= Lq) continue;  // wave-uniform
      f4 st[4];
#pragma unroll
      for (int kt = 0; kt < 4; ++kt) {
        f4 acc = {0.f, 0.f, 0.f, 0.f};
        if constexpr (k16) {
          const T* kr = Kc + (16 * kt + r) * RS + 8 * g;
          acc = mmak32<T>(cat8(*reinterpret_cast<const s4*>(kr), *reinterpret_cast<const s4*>(kr + 4)), qb16[t], acc);
        } else {
#pragma unroll
          for (int dc = 0; dc < 8; ++dc) acc = mma32(Elt<T>::to_f(Kc[(16 * kt + r) * RS + dc * 4 + g]), qb32[t][dc], acc);
        }
        st[kt] = acc;
      }
      // blocked -> -inf on the raw scores; the block max of the raw scores (sl2 > 0, checked on the host)
      mask4<0>(st[0], mcur[t][0]);
      mask4<16>(st[1], mcur[t][0]);
      mask4<0>(st[2], mcur[t][1]);
      mask4<16>(st[3], mcur[t][1]);
      float mx = -INFINITY;
#pragma unroll
      for (int kt = 0; kt < 4; ++kt)
#pragma unroll
        for (int i = 0; i < 4; ++i) mx = fmaxf(mx, st[kt][i]);
      mx = wave_max16(mx);
      // Lazy rescaling: the running max moves (and O, the row sums are rescaled by alpha) only when some query of
      // the wave sees a block max more than kLazyLog2 above it, or its first unmasked key; otherwise p is taken
      // against the stale max (p <= 2^kLazyLog2, well inside fp16 / bf16) and the rescale, its v_exp and 12
      // multiplies are skipped.  O / l and the saved LSE m + log2(l) are the same quantities either way.
      const float m_blk = mx * sl2;
      if (__any(m_blk > m_run[t] + kLazyLog2)) {   // wave-uniform; -inf + c = -inf: a first finite max moves it
        const float m_new = fmaxf(m_run[t], m_blk);
        const float alpha = ex2(m_run[t] - (m_new == -INFINITY ? 0.f : m_new));
        m_run[t] = m_new;
        o[t][0] *= alpha;
        o[t][1] *= alpha;
        if constexpr (k16) lsum[t] *= alpha;
        else l_run[t] *= alpha;
      }
      const float m_use = m_run[t] == -INFINITY ? 0.f : m_run[t];
#pragma unroll
      for (int kt = 0; kt < 4; ++kt)
#pragma unroll
        for (int i = 0; i < 4; ++i) st[kt][i] = ex2(fmaf(st[kt][i], sl2, -m_use));
      // O^T[d][q] += V^T[d][key] P^T[key][q]
      if constexpr (k16) {
#pragma unroll
        for (int pp = 0; pp < 2; ++pp) {
          const s8 pb = cat8(pack4<T>(st[2 * pp][0], st[2 * pp][1], st[2 * pp][2], st[2 * pp][3]),
                             pack4<T>(st[2 * pp + 1][0], st[2 * pp + 1][1], st[2 * pp + 1][2], st[2 * pp + 1][3]));
          lsum[t] = mmak32<T>(ones, pb, lsum[t]);
#pragma unroll
          for (int dt = 0; dt < 2; ++dt) {
            const T* vr = Vc + (32 * pp + 4 * g + (r >> 2)) * RS + dt * 16 + 4 * (r & 3);
            o[t][dt] = mmak32<T>(cat8(tr_read(vr), tr_read(vr + 16 * RS)), pb, o[t][dt]);
          }
        }
      } else {
        float rs = 0.f;
#pragma unroll
        for (int kt = 0; kt < 4; ++kt)
#pragma unroll
          for (int i = 0; i < 4; ++i) rs += st[kt][i];
        rs = wave_sum16(rs);
        l_run[t] += rs;
#pragma unroll
        for (int kt = 0; kt < 4; ++kt) {
#pragma unroll
          for (int i = 0; i < 4; ++i) {
#pragma unroll
            for (int dt = 0; dt < 2; ++dt)
              o[t][dt] = mma32(Elt<T>::to_f(Vc[(16 * kt + 4 * g + i) * RS + dt * 16 + r]), st[kt][i], o[t][dt]);
          }
        }
      }
    }
    __syncthreads();
    if (next < key_end) {
      stage_store<T>(Ks[buf ^ 1], kreg);
      stage_store<T>(Vs[buf ^ 1], vreg);
    }
    __syncthreads();
    buf ^= 1;
  }

  // epilogue: lane holds O^T[d = dt*16 + 4g + i][q = r]
  const int BH = gridDim.x;
#pragma unroll
  for (int t = 0; t < TPW; ++t) {
    if (!mrow_ok[t]) continue;
    const int qi = (w + 4 * t) * 16 + r;
    const float lt = k16 ? lsum[t][0] : l_run[t];
    if (nchunks == 1) {
      const float inv = lt > 0.f ? 1.f / lt : 0.f;
      T* orow = out + (static_cast<int64_t>(b) * Lq + qi) * (H * kD) + h * kD;
#pragma unroll
      for (int dt = 0; dt < 2; ++dt) {
        const f4 val = o[t][dt] * inv;
        if constexpr (k16) {
          *reinterpret_cast<s4*>(orow + dt * 16 + 4 * g) = pack4<T>(val[0], val[1], val[2], val[3]);
        } else {
          *reinterpret_cast<f4*>(orow + dt * 16 + 4 * g) = val;
        }
      }
      if (g == 0) lse2[static_cast<int64_t>(bh) * Lq + qi] = lt > 0.f ? m_run[t] + log2f(lt) : INFINITY;
    } else {
      const int64_t prow = (static_cast<int64_t>(c) * BH + bh) * Lq + qi;
#pragma unroll
      for (int dt = 0; dt < 2; ++dt) *reinterpret_cast<f4*>(ws_o + prow * kD + dt * 16 + 4 * g) = o[t][dt];
      if (g == 0) {
        ws_ml[2 * prow] = m_run[t];
        ws_ml[2 * prow + 1] = lt;
      }
    }
  }
}

// Combine the per-chunk partials: one thread per (b*h, q, 4 channels).
template <typename T>
__global__ void __launch_bounds__(256) mattn_combine_kernel(const float* __restrict__ ws_o,
                                                            const float* __restrict__ ws_ml, int nchunks, int BH,
                                                            int H, int Lq, T* __restrict__ out,
                                                            float* __restrict__ lse2) {
  const int64_t idx = blockIdx.x * static_cast<int64_t>(blockDim.x) + threadIdx.x;
  const int64_t total = static_cast<int64_t>(BH) * Lq * (kD / 4);
  if (idx >= total) return;
  const int part = static_cast<int>(idx % (kD / 4));
  const int64_t row = idx / (kD / 4);  // bh * Lq + q
  const int bh = static_cast<int>(row / Lq), qi = static_cast<int>(row % Lq);
  const int b = bh / H, h = bh % H;
  float M = -INFINITY;
  for (int c = 0; c < nchunks; ++c) M = fmaxf(M, ws_ml[2 * ((static_cast<int64_t>(c) * BH) * Lq + row)]);
  const float Mu = M == -INFINITY ? 0.f : M;
  float L = 0.f;
  f4 acc = {0.f, 0.f, 0.f, 0.f};
  for (int c = 0; c < nchunks; ++c) {
    const int64_t prow = static_cast<int64_t>(c) * BH * Lq + row;
    const float wgt = exp2f(ws_ml[2 * prow] - Mu);
    L += ws_ml[2 * prow + 1] * wgt;
    acc += *reinterpret_cast<const f4*>(ws_o + prow * kD + part * 4) * wgt;
  }
  const float inv = L > 0.f ? 1.f / L : 0.f;
  acc *= inv;
  T* orow = out + (static_cast<int64_t>(b) * Lq + qi) * (H * kD) + h * kD + part * 4;
  if constexpr (Elt<T>::k16) {
    *reinterpret_cast<s4*>(orow) = pack4<T>(acc[0], acc[1], acc[2], acc[3]);
  } else {
    *reinterpret_cast<f4*>(orow) = acc;
  }
  if (part == 0) lse2[row] = L > 0.f ? M + log2f(L) : INFINITY;
}

// Combine with one wave per (b*h, q): lane = 8 g + part, chunk group g takes chunks g, g + 8, ... with an online
// merge of (max, sum, 4 channels), then the 8 groups merge across lanes. The per-thread form above walks the chunks
// one after another (two passes of nchunks loads): with few rows (config 4's B = 2) it is latency-bound.
__device__ __forceinline__ void merge_part(float& m, float& l, f4& acc, float m2, float l2, const f4& a2) {
  const float mn = fmaxf(m, m2);
  if (mn == -INFINITY) return;
  const float w1 = exp2f(m - mn), w2 = exp2f(m2 - mn);
  l = l * w1 + l2 * w2;
  acc = acc * w1 + a2 * w2;
  m = mn;
}

template <typename T>
__global__ void __launch_bounds__(256) mattn_combine_wave_kernel(const float* __restrict__ ws_o,
                                                                 const float* __restrict__ ws_ml, int nchunks, int BH,
                                                                 int H, int Lq, T* __restrict__ out,
                                                                 float* __restrict__ lse2) {
  const int64_t row = blockIdx.x * 4ll + (threadIdx.x >> 6);   // bh * Lq + q, wave-uniform
  if (row >= static_cast<int64_t>(BH) * Lq) return;
  const int lane = threadIdx.x & 63, g = lane >> 3, part = lane & 7;
  float m = -INFINITY, l = 0.f;
  f4 acc = {0.f, 0.f, 0.f, 0.f};
  for (int c = g; c < nchunks; c += 8) {
    const int64_t prow = static_cast<int64_t>(c) * BH * Lq + row;
    const float2 ml = *reinterpret_cast<const float2*>(ws_ml + 2 * prow);
    merge_part(m, l, acc, ml.x, ml.y, *reinterpret_cast<const f4*>(ws_o + prow * kD + part * 4));
  }
#pragma unroll
  for (int o = 8; o < 64; o <<= 1) {
    const float m2 = __shfl_xor(m, o), l2 = __shfl_xor(l, o);
    f4 a2;
    for (int i = 0; i < 4; ++i) a2[i] = __shfl_xor(acc[i], o);
    merge_part(m, l, acc, m2, l2, a2);
  }
  if (g != 0) return;
  const int bh = static_cast<int>(row / Lq), qi = static_cast<int>(row % Lq);
  const int b = bh / H, h = bh % H;
  const float inv = l > 0.f ? 1.f / l : 0.f;
  acc *= inv;
  T* orow = out + (static_cast<int64_t>(b) * Lq + qi) * (H * kD) + h * kD + part * 4;
  if constexpr (Elt<T>::k16) {
    *reinterpret_cast<s4*>(orow) = pack4<T>(acc[0], acc[1], acc[2], acc[3]);
  } else {
    *reinterpret_cast<f4*>(orow) = acc;
  }
  if (part == 0) lse2[row] = l > 0.f ? m + log2f(l) : INFINITY;
}

// ----------------------------------------------------------------------------------------------
// 3. masked attention backward
// ----------------------------------------------------------------------------------------------
// grid (B*H, nchunks), 256 threads.  Per 64-key block wave w owns key tile w: dK^T and dV^T stay in
// registers; S = Q K^T is computed with the query on rows so that P and dS (C layout) are directly
// the B operands of dV^T += dO^T P and dK^T += Q^T dS; dQ^T += K^T dS^T needs dS^T, transposed
// through a per-wave 16x16 LDS scratch.  With NTR > 0 (Lq <= 16 * NTR) each wave keeps its dQ^T in
// registers over the whole chunk and the four waves are summed through LDS once at the end; with
// NTR == -1 (Lq <= 208: config 4's Q = 200) each wave adds its tiles' dQ^T into its own LDS copy with plain
// read-modify-writes (no two waves touch one copy) and the four copies are summed at the end; with
// NTR == 0 (more queries) each tile's dQ^T goes to LDS float atomics (~190 cycles per wave-instruction
// on gfx950, the reason for the other two paths).  Chunks are summed by a reduce pass (deterministic).
template <typename T, int NTR>
__global__ void __launch_bounds__(256, NTR > 8 ? 2 : 1) mattn_bwd_kernel(
    const T* __restrict__ q, const T* __restrict__ k, const T* __restrict__ v, const uint32_t* __restrict__ bits,
    const T* __restrict__ out, const T* __restrict__ dout, const float* __restrict__ lse2, int Lq, int Lk, int H,
    int qs, int kvs, int nw, float sl2, float scale, int chunk_len, int Lqp, T* __restrict__ dq,
    T* __restrict__ dk, T* __restrict__ dv, float* __restrict__ ws_dq, int xmap) {
  constexpr bool k16 = Elt<T>::k16;
  constexpr int RS = KVImage<T>::RS;
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  // carve: Qs, dOs [Lqp][RS] T | Ks, Vs [64][RS] T | lse, delta [Lqp] f32 | mw [2][Lqp] u32 (word 0 / 1 of the block,
  //        keys past the chunk set) | scr [4][16][17] f32 | dQacc [Lqp][kD] f32
  T* Qs = reinterpret_cast<T*>(smem);
  T* dOs = Qs + Lqp * RS;
  T* Ks = dOs + Lqp * RS;
  T* Vs = Ks + 64 * RS;
  size_t off = (reinterpret_cast<unsigned char*>(Vs + 64 * RS) - smem + 15) & ~size_t(15);
  float* lse_s = reinterpret_cast<float*>(smem + off);
  float* del_s = lse_s + Lqp;
  uint32_t* mw = reinterpret_cast<uint32_t*>(del_s + Lqp);
  float* scr = reinterpret_cast<float*>(mw + 2 * Lqp);
  float* dqa = scr + 4 * 16 * 17;
  const int dq_elems = NTR > 0 ? Lqp * kDQ : Lqp * kD;   // register-dQ modes: padded rows (kDQ)

  int bh, c;
  mattn_block(H, xmap, bh, c);
  const int b = bh / H, h = bh % H;
  const int nchunks = gridDim.y;
  const int key_begin = c * chunk_len;
  const int key_end = min(Lk, key_begin + chunk_len);
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6, g = lane >> 4, r = lane & 15;
  const int64_t kvrow0 = static_cast<int64_t>(b) * Lk;
  const int NT = Lqp / 16;
  const int HD = H * kD;

  // stage Q, dO (rows >= Lq zero), lse, delta; clear dQ accumulator.  16-bit operands move in 16-byte pieces (the
  // 72-byte LDS rows take them as two 8-byte halves); delta = sum_d O dO in d order from a thread's four pieces
  if constexpr (k16) {
    for (int idx = threadIdx.x; idx < Lqp * 4; idx += 256) {
      const int qi = idx >> 2, part = idx & 3;
      f4 qv = {0.f, 0.f, 0.f, 0.f}, gv = qv;
      if (qi < Lq) {
        qv = *reinterpret_cast<const f4*>(q + (static_cast<int64_t>(b) * Lq + qi) * qs + h * kD + part * 8);
        gv = *reinterpret_cast<const f4*>(dout + (static_cast<int64_t>(b) * Lq + qi) * HD + h * kD + part * 8);
      }
      const s4* qh = reinterpret_cast<const s4*>(&qv);
      const s4* gh = reinterpret_cast<const s4*>(&gv);
      s4* qd = reinterpret_cast<s4*>(Qs + qi * RS + part * 8);
      s4* gd = reinterpret_cast<s4*>(dOs + qi * RS + part * 8);
      qd[0] = qh[0]; qd[1] = qh[1];
      gd[0] = gh[0]; gd[1] = gh[1];
    }
    for (int idx = threadIdx.x; idx < dq_elems / 4; idx += 256) reinterpret_cast<f4*>(dqa)[idx] = f4{0.f, 0.f, 0.f, 0.f};
  } else {
    for (int idx = threadIdx.x; idx < Lqp * kD; idx += 256) {
      const int qi = idx / kD, d = idx % kD;
      T qv = Elt<T>::from_f(0.f), gv = Elt<T>::from_f(0.f);
      if (qi < Lq) {
        qv = q[(static_cast<int64_t>(b) * Lq + qi) * qs + h * kD + d];
        gv = dout[(static_cast<int64_t>(b) * Lq + qi) * HD + h * kD + d];
      }
      Qs[qi * RS + d] = qv;
      dOs[qi * RS + d] = gv;
      dqa[idx] = 0.f;
    }
    for (int idx = Lqp * kD + threadIdx.x; idx < dq_elems; idx += 256) dqa[idx] = 0.f;   // the padding
  }
  for (int qi = threadIdx.x; qi < Lqp; qi += 256) {
    float dl = 0.f, ls = INFINITY;
    if (qi < Lq) {
      const T* orow = out + (static_cast<int64_t>(b) * Lq + qi) * HD + h * kD;
      const T* grow = dout + (static_cast<int64_t>(b) * Lq + qi) * HD + h * kD;
      if constexpr (k16) {
        f4 ov[4], gv[4];
#pragma unroll
        for (int p = 0; p < 4; ++p) {
          ov[p] = *reinterpret_cast<const f4*>(orow + p * 8);
          gv[p] = *reinterpret_cast<const f4*>(grow + p * 8);
        }
#pragma unroll
        for (int p = 0; p < 4; ++p) {
          const T* oe = reinterpret_cast<const T*>(&ov[p]);
          const T* ge = reinterpret_cast<const T*>(&gv[p]);
#pragma unroll
          for (int e = 0; e < 8; ++e) dl += Elt<T>::to_f(oe[e]) * Elt<T>::to_f(ge[e]);
        }
      } else {
        for (int d = 0; d < kD; ++d) dl += Elt<T>::to_f(orow[d]) * Elt<T>::to_f(grow[d]);
      }
      ls = lse2[static_cast<int64_t>(bh) * Lq + qi];
    }
    del_s[qi] = -dl;   // negated: the pair updates add them
    lse_s[qi] = -ls;
  }

  float* myscr = scr + w * 16 * 17;
  f4 dqacc[NTR > 0 ? NTR : 1][2];
#pragma unroll
  for (int qt = 0; qt < (NTR > 0 ? NTR : 1); ++qt) dqacc[qt][0] = dqacc[qt][1] = f4{0.f, 0.f, 0.f, 0.f};
  float* dqw = dqa + (NTR < 0 ? w * Lqp * kD : 0);   // this wave's dQ copy (NTR == -1)
  if constexpr (NTR < 0) {
    for (int idx = threadIdx.x; idx < 3 * Lqp * kD; idx += 256) dqa[Lqp * kD + idx] = 0.f;   // copies 1..3
  }
  // software pipeline: the next key block's K / V rows and mask words are loaded into registers while the
  // current block is computed (one LDS image; it is rewritten after the barrier that ends its use)
  constexpr int kMaxMwPerThread = 2;   // Lqp <= 512
  f4 kreg[2], vreg[2];
  uint32_t mreg[kMaxMwPerThread][2];
  // (no exec branches around the loads, so the compiler's wait counting leaves them in flight: rows past the chunk
  // repeat its last row, those keys being masked; mask words load at clamped addresses and a query past Lq or a word
  // past the row is overridden where the words are staged)
  auto prefetch = [&](int kb) {
    stage_load<T, true>(k, kvrow0 + kb, key_end - kb, kvs, h * kD, kreg);
    stage_load<T, true>(v, kvrow0 + kb, key_end - kb, kvs, h * kD, vreg);
    const int w1 = min((kb >> 5) + 1, nw - 1);
#pragma unroll
    for (int u = 0; u < kMaxMwPerThread; ++u) {
      const uint32_t* mr = bits + (static_cast<int64_t>(b) * Lq + min(static_cast<int>(threadIdx.x) + 256 * u, Lq - 1)) * nw;
      mreg[u][0] = mr[kb >> 5];
      mreg[u][1] = mr[w1];
    }
  };
  if (key_begin < key_end) prefetch(key_begin);
  for (int kb0 = key_begin; kb0 < key_end; kb0 += 64) {
    __syncthreads();  // previous block's images fully consumed (and the prologue staged)
    stage_store<T>(Ks, kreg);
    stage_store<T>(Vs, vreg);
    const int kvalid = key_end - kb0;
    {
      const uint32_t x0 = kvalid >= 32 ? 0u : (0xffffffffu << (kvalid & 31));
      const uint32_t x1 = kvalid >= 64 ? 0u : (kvalid <= 32 ? 0xffffffffu : (0xffffffffu << ((kvalid - 32) & 31)));
      const uint32_t xw = (kb0 >> 5) + 1 < nw ? 0u : 0xffffffffu;  // no second word: keys past Lk
#pragma unroll
      for (int u = 0; u < kMaxMwPerThread; ++u) {
        const int qi = threadIdx.x + 256 * u;
        if (qi < Lqp) {
          const uint32_t xr = qi < Lq ? 0u : 0xffffffffu;
          mw[qi] = ~(mreg[u][0] | x0 | xr);   // inverted: bit set = key visible
          mw[Lqp + qi] = ~(mreg[u][1] | x1 | xw | xr);
        }
      }
    }
    __syncthreads();
    if (kb0 + 64 < key_end) prefetch(kb0 + 64);   // in flight during this block's MFMAs
    const int koff = 16 * w + r;  // this lane's key (column) within the block
    if (16 * w >= kvalid) continue;  // whole tile beyond the chunk (wave-uniform); barriers are at loop top

    // per-key-tile operands: K, V as B[k = d][col = key] (16-bit: d = 8g + j, one 16x16x32 over the head dim)
    s8 kb16, vb16;
    float kb32[8], vb32[8];
    if constexpr (k16) {
      const T* kr = Ks + koff * RS + 8 * g;
      const T* vr = Vs + koff * RS + 8 * g;
      kb16 = cat8(*reinterpret_cast<const s4*>(kr), *reinterpret_cast<const s4*>(kr + 4));
      vb16 = cat8(*reinterpret_cast<const s4*>(vr), *reinterpret_cast<const s4*>(vr + 4));
    } else {
#pragma unroll
      for (int dc = 0; dc < 8; ++dc) {
        kb32[dc] = Elt<T>::to_f(Ks[koff * RS + dc * 4 + g]);
        vb32[dc] = Elt<T>::to_f(Vs[koff * RS + dc * 4 + g]);
      }
    }
    f4 dkacc[2] = {f4{0.f, 0.f, 0.f, 0.f}, f4{0.f, 0.f, 0.f, 0.f}};
    f4 dvacc[2] = {f4{0.f, 0.f, 0.f, 0.f}, f4{0.f, 0.f, 0.f, 0.f}};
    const uint32_t* mwsel = mw + (koff >> 5) * Lqp;  // wave-uniform word of the block
    const uint32_t bit = koff & 31;
    const bool key_ok = koff < kvalid;

    // dV^T += dO^T P ; dK^T += Q^T dS (A[row d][k = q]).  16-bit: two query tiles per 16x16x32 (K = 32 queries,
    // element j < 4 of a lane's fragments from the first tile's query 4g + j, j >= 4 from the second's), one tile on
    // 16x16x16 for an odd tail
    auto dvdk2 = [&](int qa, s4 pa, s4 sa, int qb, s4 pb, s4 sb) {
#pragma unroll
      for (int dt = 0; dt < 2; ++dt) {
        const int ra = (qa * 16 + 4 * g + (r >> 2)) * RS + dt * 16 + 4 * (r & 3);
        const int rb = (qb * 16 + 4 * g + (r >> 2)) * RS + dt * 16 + 4 * (r & 3);
        dvacc[dt] = mmak32<T>(cat8(tr_read(dOs + ra), tr_read(dOs + rb)), cat8(pa, pb), dvacc[dt]);
        dkacc[dt] = mmak32<T>(cat8(tr_read(Qs + ra), tr_read(Qs + rb)), cat8(sa, sb), dkacc[dt]);
      }
    };
    auto dvdk1 = [&](int qa, s4 pa, s4 sa) {
#pragma unroll
      for (int dt = 0; dt < 2; ++dt) {
        const int ro = (qa * 16 + 4 * g + (r >> 2)) * RS + dt * 16 + 4 * (r & 3);
        dvacc[dt] = mma16<T>(tr_read(dOs + ro), pa, dvacc[dt]);
        dkacc[dt] = mma16<T>(tr_read(Qs + ro), sa, dkacc[dt]);
      }
    };

    // one 16-query tile against this wave's 16 keys; dQ^T contributions accumulate into dqt; 16-bit: P and dS
    // packed into pb / sb for dvdk (f32: dV / dK accumulated here)
    auto tile = [&](const int qt, f4* dqt, s4& pbo, s4& sbo) {
      f4 s = {0.f, 0.f, 0.f, 0.f}, dp = {0.f, 0.f, 0.f, 0.f};
      if constexpr (k16) {
        const T* qr = Qs + (qt * 16 + r) * RS + 8 * g;
        const T* gr = dOs + (qt * 16 + r) * RS + 8 * g;
        s = mmak32<T>(cat8(*reinterpret_cast<const s4*>(qr), *reinterpret_cast<const s4*>(qr + 4)), kb16, s);
        dp = mmak32<T>(cat8(*reinterpret_cast<const s4*>(gr), *reinterpret_cast<const s4*>(gr + 4)), vb16, dp);
      } else {
#pragma unroll
        for (int dc = 0; dc < 8; ++dc) {
          s = mma32(Elt<T>::to_f(Qs[(qt * 16 + r) * RS + dc * 4 + g]), kb32[dc], s);
          dp = mma32(Elt<T>::to_f(dOs[(qt * 16 + r) * RS + dc * 4 + g]), vb32[dc], dp);
        }
      }
      // C layout: [q = qt*16 + 4g + i][key = koff]; the four queries' mask words, LSE and delta in one 16-B read each
      const int q0 = qt * 16 + 4 * g;
      const uint4 mq = *reinterpret_cast<const uint4*>(mwsel + q0);
      const f4 nlq = *reinterpret_cast<const f4*>(lse_s + q0);   // -LSE
      const f4 ndq = *reinterpret_cast<const f4*>(del_s + q0);   // -delta
      const uint32_t mqa[4] = {mq.x, mq.y, mq.z, mq.w};
      f4 p, ds;
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const float pv = keep_bit(mqa[i], bit, ex2(fmaf(s[i], sl2, nlq[i])));
        p[i] = pv;
        ds[i] = pv * (dp[i] + ndq[i]);
      }
      if constexpr (k16) {
        pbo = pack4<T>(p[0], p[1], p[2], p[3]);
        sbo = pack4<T>(ds[0], ds[1], ds[2], ds[3]);
      } else {
#pragma unroll
        for (int i = 0; i < 4; ++i) {
#pragma unroll
          for (int dt = 0; dt < 2; ++dt) {
            const int ro = (qt * 16 + 4 * g + i) * RS + dt * 16 + r;
            dvacc[dt] = mma32(Elt<T>::to_f(dOs[ro]), p[i], dvacc[dt]);
            dkacc[dt] = mma32(Elt<T>::to_f(Qs[ro]), ds[i], dkacc[dt]);
          }
        }
      }
      // dQ^T[d][q] += K^T[d][key] dS^T[key][q]: transpose dS through the wave's scratch
#pragma unroll
      for (int i = 0; i < 4; ++i) myscr[(4 * g + i) * 17 + r] = ds[i];  // scr[q][key]
      __builtin_amdgcn_wave_barrier();
      float dst4[4];
#pragma unroll
      for (int j = 0; j < 4; ++j) dst4[j] = myscr[r * 17 + 4 * g + j];  // dS^T[key = 4g+j][q = r]
      __builtin_amdgcn_wave_barrier();
      if constexpr (k16) {
        const s4 sb = pack4<T>(dst4[0], dst4[1], dst4[2], dst4[3]);
#pragma unroll
        for (int dt = 0; dt < 2; ++dt) {
          const s4 ka = tr_read(Ks + (16 * w + 4 * g + (r >> 2)) * RS + dt * 16 + 4 * (r & 3));
          dqt[dt] = mma16<T>(ka, sb, dqt[dt]);
        }
      } else {
#pragma unroll
        for (int i = 0; i < 4; ++i) {
#pragma unroll
          for (int dt = 0; dt < 2; ++dt)
            dqt[dt] = mma32(Elt<T>::to_f(Ks[(16 * w + 4 * g + i) * RS + dt * 16 + r]), dst4[i], dqt[dt]);
        }
      }
    };
    s4 ppend = {0, 0, 0, 0}, spend = {0, 0, 0, 0};  // 16-bit: an even tile's P / dS waiting for its pair
    auto tile_done = [&](int qt, s4 pb, s4 sb) {
      if constexpr (k16) {
        if (qt & 1) dvdk2(qt - 1, ppend, spend, qt, pb, sb);
        else { ppend = pb; spend = sb; }
      }
    };
    if constexpr (NTR > 0) {
      // dQ stays in registers across every key block of the chunk (Lqp <= 16 * NTR)
#pragma unroll
      for (int qt = 0; qt < NTR; ++qt)
        if (qt < NT) {
          s4 pb, sb;
          tile(qt, dqacc[qt], pb, sb);
          tile_done(qt, pb, sb);
        }
    } else {
      for (int qt = 0; qt < NT; ++qt) {
        f4 dqt[2] = {f4{0.f, 0.f, 0.f, 0.f}, f4{0.f, 0.f, 0.f, 0.f}};
        s4 pb, sb;
        tile(qt, dqt, pb, sb);
        tile_done(qt, pb, sb);
        // lane holds dQ^T[d = dt*16 + 4g + i][q = qt*16 + r]
        if constexpr (NTR < 0) {
#pragma unroll
          for (int dt = 0; dt < 2; ++dt) {
            f4* dst = reinterpret_cast<f4*>(&dqw[(qt * 16 + r) * kD + dt * 16 + 4 * g]);
            *dst = *dst + dqt[dt];
          }
        } else {
#pragma unroll
          for (int dt = 0; dt < 2; ++dt)
#pragma unroll
            for (int i = 0; i < 4; ++i) atomicAdd(&dqa[(qt * 16 + r) * kD + dt * 16 + 4 * g + i], dqt[dt][i]);
        }
      }
    }
    if constexpr (k16) {
      if (NT & 1) dvdk1(NT - 1, ppend, spend);
    }
    // write dK, dV for this key tile: lane holds [d = dt*16 + 4g + i][key = koff]
    if (key_ok) {
      const int64_t krow = (kvrow0 + kb0 + koff) * HD + h * kD;
#pragma unroll
      for (int dt = 0; dt < 2; ++dt) {
        const f4 kk = dkacc[dt] * scale;
        const f4 vv = dvacc[dt];
        if constexpr (k16) {
          *reinterpret_cast<s4*>(dk + krow + dt * 16 + 4 * g) = pack4<T>(kk[0], kk[1], kk[2], kk[3]);
          *reinterpret_cast<s4*>(dv + krow + dt * 16 + 4 * g) = pack4<T>(vv[0], vv[1], vv[2], vv[3]);
        } else {
          *reinterpret_cast<f4*>(dk + krow + dt * 16 + 4 * g) = kk;
          *reinterpret_cast<f4*>(dv + krow + dt * 16 + 4 * g) = vv;
        }
      }
    }
  }
  if constexpr (NTR > 0) {
    // sum the four waves' register dQ^T into dqa, one wave at a time (plain LDS read-modify-write)
    // lane holds dQ^T[d = dt*16 + 4g + i][q = qt*16 + r]; rows of kDQ floats
    for (int ww = 0; ww < 4; ++ww) {
      __syncthreads();
      if (w == ww) {
#pragma unroll
        for (int qt = 0; qt < NTR; ++qt) {
          if (qt < NT) {
#pragma unroll
            for (int dt = 0; dt < 2; ++dt)
#pragma unroll
              for (int i = 0; i < 4; ++i) dqa[(qt * 16 + r) * kDQ + dt * 16 + 4 * g + i] += dqacc[qt][dt][i];
          }
        }
      }
    }
  }
  __syncthreads();
  // dQ partial for this chunk
  const int BH = gridDim.x;
  for (int idx = threadIdx.x; idx < Lq * kD; idx += 256) {
    const int qi = idx / kD, d = idx % kD;
    float sum = dqa[NTR > 0 ? qi * kDQ + d : idx];
    if constexpr (NTR < 0) sum = ((sum + dqa[Lqp * kD + idx]) + dqa[2 * Lqp * kD + idx]) + dqa[3 * Lqp * kD + idx];
    const float val = sum * scale;
    if (nchunks == 1)
      dq[(static_cast<int64_t>(b) * Lq + qi) * HD + h * kD + d] = Elt<T>::from_f(val);
    else
      ws_dq[((static_cast<int64_t>(c) * BH + bh) * Lq + qi) * kD + d] = val;
  }
}

// Two key tiles per wave (16-bit operands, dQ in registers: Lq <= 16 * NTR): per 128-key block wave w owns keys
// 32w .. 32w + 31 (tile a: 32w + r, tile b: 32w + 16 + r).  Everything a query tile needs -- its Q / dO fragments,
// mask words (both tiles' keys sit in one word), LSE, delta and the dO^T / Q^T fragments of the dV / dK products --
// is read from LDS once for both key tiles, and dQ^T += K^T dS^T runs as one 16x16x32 product over the 32 keys
// instead of four 16x16x16 ones.  The dS transpose goes through a 20-float-pitch scratch, so a lane reads its four
// transposed values with one 16-byte read.  Same arithmetic per element as mattn_bwd_kernel (the dQ^T sum over a
// block's keys is one MFMA chain in another key order).
template <typename T, int NTR>
__global__ void __launch_bounds__(256, 2) mattn_bwd2_kernel(
    const T* __restrict__ q, const T* __restrict__ k, const T* __restrict__ v, const uint32_t* __restrict__ bits,
    const T* __restrict__ out, const T* __restrict__ dout, const float* __restrict__ lse2, int Lq, int Lk, int H,
    int qs, int kvs, int nw, float sl2, float scale, int chunk_len, int Lqp, T* __restrict__ dq,
    T* __restrict__ dk, T* __restrict__ dv, float* __restrict__ ws_dq, int xmap) {
  static_assert(Elt<T>::k16 && NTR > 0, "16-bit operands, register dQ");
  constexpr int RS = KVImage<T>::RS;
  constexpr int SP = 20;  // transpose scratch pitch (floats): 16-byte aligned rows, conflict-free column writes
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  // carve: Qs, dOs [Lqp][RS] T | Ks, Vs [2][128][RS] T | lse, delta [Lqp] f32 | mw [2][4][Lqp] u32 | scr [4][16][SP]
  //        f32 (x2: tiles a / b); dQacc [Lqp][kD] f32 over the K / V images once the key loop is done (two
  //        workgroups per CU: 67.7 KB at Lqp = 112)
  T* Qs = reinterpret_cast<T*>(smem);
  T* dOs = Qs + Lqp * RS;
  T* Ks2 = dOs + Lqp * RS;
  T* Vs2 = Ks2 + 2 * 128 * RS;
  size_t off = (reinterpret_cast<unsigned char*>(Vs2 + 2 * 128 * RS) - smem + 15) & ~size_t(15);
  float* lse_s = reinterpret_cast<float*>(smem + off);
  float* del_s = lse_s + Lqp;
  uint32_t* mw2 = reinterpret_cast<uint32_t*>(del_s + Lqp);
  float* scr = reinterpret_cast<float*>(mw2 + 8 * Lqp);
  float* dqa = reinterpret_cast<float*>(Ks2);   // 16-byte aligned: Qs and dOs are Lqp * RS * 2 bytes, Lqp % 16 == 0

  int bh, c;
  mattn_block(H, xmap, bh, c);
  const int b = bh / H, h = bh % H;
  const int nchunks = gridDim.y;
  const int key_begin = c * chunk_len;
  const int key_end = min(Lk, key_begin + chunk_len);
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6, g = lane >> 4, r = lane & 15;
  const int64_t kvrow0 = static_cast<int64_t>(b) * Lk;
  const int NT = Lqp / 16;
  const int HD = H * kD;

  // stage Q, dO (rows >= Lq zero), lse, delta (as mattn_bwd_kernel)
  for (int idx = threadIdx.x; idx < Lqp * 4; idx += 256) {
    const int qi = idx >> 2, part = idx & 3;
    f4 qv = {0.f, 0.f, 0.f, 0.f}, gv = qv;
    if (qi < Lq) {
      qv = *reinterpret_cast<const f4*>(q + (static_cast<int64_t>(b) * Lq + qi) * qs + h * kD + part * 8);
      gv = *reinterpret_cast<const f4*>(dout + (static_cast<int64_t>(b) * Lq + qi) * HD + h * kD + part * 8);
    }
    const s4* qh = reinterpret_cast<const s4*>(&qv);
    const s4* gh = reinterpret_cast<const s4*>(&gv);
    s4* qd = reinterpret_cast<s4*>(Qs + qi * RS + part * 8);
    s4* gd = reinterpret_cast<s4*>(dOs + qi * RS + part * 8);
    qd[0] = qh[0]; qd[1] = qh[1];
    gd[0] = gh[0]; gd[1] = gh[1];
  }
  for (int qi = threadIdx.x; qi < Lqp; qi += 256) {
    float dl = 0.f, ls = INFINITY;
    if (qi < Lq) {
      const T* orow = out + (static_cast<int64_t>(b) * Lq + qi) * HD + h * kD;
      const T* grow = dout + (static_cast<int64_t>(b) * Lq + qi) * HD + h * kD;
      f4 ov[4], gv[4];
#pragma unroll
      for (int p = 0; p < 4; ++p) {
        ov[p] = *reinterpret_cast<const f4*>(orow + p * 8);
        gv[p] = *reinterpret_cast<const f4*>(grow + p * 8);
      }
#pragma unroll
      for (int p = 0; p < 4; ++p) {
        const T* oe = reinterpret_cast<const T*>(&ov[p]);
        const T* ge = reinterpret_cast<const T*>(&gv[p]);
#pragma unroll
        for (int e = 0; e < 8; ++e) dl += Elt<T>::to_f(oe[e]) * Elt<T>::to_f(ge[e]);
      }
      ls = lse2[static_cast<int64_t>(bh) * Lq + qi];
    }
    del_s[qi] = -dl;   // negated: the pair updates add them
    lse_s[qi] = -ls;
  }

  float* myscr = scr + w * 2 * 16 * SP;   // tile a's [16][SP], then tile b's
  f4 dqacc[NTR][2];
#pragma unroll
  for (int qt = 0; qt < NTR; ++qt) dqacc[qt][0] = dqacc[qt][1] = f4{0.f, 0.f, 0.f, 0.f};

  // the next 128-key block's K / V rows (two 64-row halves) and mask words (4 per query) in registers
  constexpr int kMaxMwPerThread = 1;   // Lqp <= 256 (the kernel runs at Lqp <= 128)
  f4 kreg[2][2], vreg[2][2];
  uint32_t mreg[kMaxMwPerThread][4];
  auto prefetch = [&](int kb) {
#pragma unroll
    for (int hf = 0; hf < 2; ++hf) {
      const int kh = min(kb + 64 * hf, key_end - 1);   // a half past the chunk repeats its last row (masked)
      stage_load<T, true>(k, kvrow0 + kh, key_end - kh, kvs, h * kD, kreg[hf]);
      stage_load<T, true>(v, kvrow0 + kh, key_end - kh, kvs, h * kD, vreg[hf]);
    }
#pragma unroll
    for (int u = 0; u < kMaxMwPerThread; ++u) {
      const uint32_t* mr = bits + (static_cast<int64_t>(b) * Lq + min(static_cast<int>(threadIdx.x) + 256 * u, Lq - 1)) * nw;
#pragma unroll
      for (int t = 0; t < 4; ++t) mreg[u][t] = mr[min((kb >> 5) + t, nw - 1)];
    }
  };
  if (key_begin < key_end) prefetch(key_begin);
  int buf = 0;
  for (int kb0 = key_begin; kb0 < key_end; kb0 += 128, buf ^= 1) {
    // two images: this block's was last read two blocks ago, before the previous block's barrier
    T* Ks = Ks2 + buf * 128 * RS;
    T* Vs = Vs2 + buf * 128 * RS;
    uint32_t* mw = mw2 + buf * 4 * Lqp;
    stage_store<T>(Ks, kreg[0]);
    stage_store<T>(Ks + 64 * RS, kreg[1]);
    stage_store<T>(Vs, vreg[0]);
    stage_store<T>(Vs + 64 * RS, vreg[1]);
    const int kvalid = key_end - kb0;
#pragma unroll
    for (int u = 0; u < kMaxMwPerThread; ++u) {
      const int qi = threadIdx.x + 256 * u;
      if (qi < Lqp) {
        const uint32_t xr = qi < Lq ? 0u : 0xffffffffu;
#pragma unroll
        for (int t = 0; t < 4; ++t) {
          // keys 32t .. 32t + 31 of the block: those past the chunk (or past Lk: no such word) set
          const int kv = kvalid - 32 * t;
          const uint32_t xk = kv >= 32 ? 0u : (kv <= 0 ? 0xffffffffu : (0xffffffffu << (kv & 31)));
          const uint32_t xw = (kb0 >> 5) + t < nw ? 0u : 0xffffffffu;
          mw[t * Lqp + qi] = ~(mreg[u][t] | xk | xw | xr);   // inverted: bit set = key visible
        }
      }
    }
    __syncthreads();
    if (kb0 + 128 < key_end) prefetch(kb0 + 128);   // in flight during this block's MFMAs
    if (32 * w >= kvalid) continue;                 // both of this wave's tiles past the chunk (wave-uniform)
    const int ka = 32 * w + r, kb = ka + 16;        // this lane's keys (columns) within the block

    // K, V as B[k = d][col = key] for both tiles
    const T* kra = Ks + ka * RS + 8 * g;
    const T* krb = Ks + kb * RS + 8 * g;
    const T* vra = Vs + ka * RS + 8 * g;
    const T* vrb = Vs + kb * RS + 8 * g;
    const s8 kba = cat8(*reinterpret_cast<const s4*>(kra), *reinterpret_cast<const s4*>(kra + 4));
    const s8 kbb = cat8(*reinterpret_cast<const s4*>(krb), *reinterpret_cast<const s4*>(krb + 4));
    const s8 vba = cat8(*reinterpret_cast<const s4*>(vra), *reinterpret_cast<const s4*>(vra + 4));
    const s8 vbb = cat8(*reinterpret_cast<const s4*>(vrb), *reinterpret_cast<const s4*>(vrb + 4));
    // K^T fragments of dQ^T += K^T dS^T (A[row d][k = key], the 32 keys in the order tile a 4g+j, tile b 4g+j)
    s8 kta[2];
#pragma unroll
    for (int dt = 0; dt < 2; ++dt)
      kta[dt] = cat8(tr_read(Ks + (32 * w + 4 * g + (r >> 2)) * RS + dt * 16 + 4 * (r & 3)),
                     tr_read(Ks + (32 * w + 16 + 4 * g + (r >> 2)) * RS + dt * 16 + 4 * (r & 3)));
    f4 dka[2] = {f4{0.f, 0.f, 0.f, 0.f}, f4{0.f, 0.f, 0.f, 0.f}}, dkb[2] = {dka[0], dka[1]};
    f4 dva[2] = {dka[0], dka[1]}, dvb[2] = {dka[0], dka[1]};
    const uint32_t* mwsel = mw + w * Lqp;   // keys 32w .. 32w + 31: one word; tile a bit r, tile b bit 16 + r

    // one query tile against the wave's 32 keys: P, dS of both tiles (packed for dV / dK), dQ^T
    auto tile = [&](const int qt, f4* dqt, s4& pa, s4& sa, s4& pb, s4& sb) {
      const T* qr = Qs + (qt * 16 + r) * RS + 8 * g;
      const T* gr = dOs + (qt * 16 + r) * RS + 8 * g;
      const s8 qf = cat8(*reinterpret_cast<const s4*>(qr), *reinterpret_cast<const s4*>(qr + 4));
      const s8 gf = cat8(*reinterpret_cast<const s4*>(gr), *reinterpret_cast<const s4*>(gr + 4));
      const f4 z = {0.f, 0.f, 0.f, 0.f};
      const f4 s_a = mmak32<T>(qf, kba, z), s_b = mmak32<T>(qf, kbb, z);
      const f4 dp_a = mmak32<T>(gf, vba, z), dp_b = mmak32<T>(gf, vbb, z);
      const int q0 = qt * 16 + 4 * g;
      const uint4 mq = *reinterpret_cast<const uint4*>(mwsel + q0);
      const f4 nlq = *reinterpret_cast<const f4*>(lse_s + q0);   // -LSE
      const f4 ndq = *reinterpret_cast<const f4*>(del_s + q0);   // -delta
      const uint32_t mqa[4] = {mq.x, mq.y, mq.z, mq.w};
      // scalar VALU (packed f32 ops cost more than their scalar pairs beside MFMAs: MI355X_MICROARCH.md issue costs)
      f4 P_a, S_a, P_b, S_b;
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const float pva = keep_bit(mqa[i], r, ex2(fmaf(s_a[i], sl2, nlq[i])));
        const float pvb = keep_bit(mqa[i], 16 + r, ex2(fmaf(s_b[i], sl2, nlq[i])));
        P_a[i] = pva;
        S_a[i] = pva * (dp_a[i] + ndq[i]);
        P_b[i] = pvb;
        S_b[i] = pvb * (dp_b[i] + ndq[i]);
      }
      pa = pack4<T>(P_a[0], P_a[1], P_a[2], P_a[3]);
      sa = pack4<T>(S_a[0], S_a[1], S_a[2], S_a[3]);
      pb = pack4<T>(P_b[0], P_b[1], P_b[2], P_b[3]);
      sb = pack4<T>(S_b[0], S_b[1], S_b[2], S_b[3]);
      // dS^T through the scratch: [q][key] rows of pitch SP, read back as dS^T[key = 4g + j][q = r]
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        myscr[(4 * g + i) * SP + r] = S_a[i];
        myscr[16 * SP + (4 * g + i) * SP + r] = S_b[i];
      }
      __builtin_amdgcn_wave_barrier();
      // the lane needs dS[q = r][key = 4g + j]: row r, columns 4g .. 4g + 3 of the [q][key] image, one 16-byte read
      const f4 ta = *reinterpret_cast<const f4*>(myscr + r * SP + 4 * g);
      const f4 tb = *reinterpret_cast<const f4*>(myscr + 16 * SP + r * SP + 4 * g);
      __builtin_amdgcn_wave_barrier();
      const s8 sbt = cat8(pack4<T>(ta[0], ta[1], ta[2], ta[3]), pack4<T>(tb[0], tb[1], tb[2], tb[3]));
#pragma unroll
      for (int dt = 0; dt < 2; ++dt) dqt[dt] = mmak32<T>(kta[dt], sbt, dqt[dt]);
    };
    // dV^T += dO^T P, dK^T += Q^T dS for both key tiles over a pair of query tiles (the dO^T / Q^T fragments once)
    auto dvdk2 = [&](int qa, s4 pa_a, s4 sa_a, s4 pa_b, s4 sa_b, int qb, s4 pb_a, s4 sb_a, s4 pb_b, s4 sb_b) {
#pragma unroll
      for (int dt = 0; dt < 2; ++dt) {
        const int ra = (qa * 16 + 4 * g + (r >> 2)) * RS + dt * 16 + 4 * (r & 3);
        const int rb = (qb * 16 + 4 * g + (r >> 2)) * RS + dt * 16 + 4 * (r & 3);
        const s8 go = cat8(tr_read(dOs + ra), tr_read(dOs + rb));
        const s8 qo = cat8(tr_read(Qs + ra), tr_read(Qs + rb));
        dva[dt] = mmak32<T>(go, cat8(pa_a, pb_a), dva[dt]);
        dvb[dt] = mmak32<T>(go, cat8(pa_b, pb_b), dvb[dt]);
        dka[dt] = mmak32<T>(qo, cat8(sa_a, sb_a), dka[dt]);
        dkb[dt] = mmak32<T>(qo, cat8(sa_b, sb_b), dkb[dt]);
      }
    };
    auto dvdk1 = [&](int qa, s4 pa_a, s4 sa_a, s4 pa_b, s4 sa_b) {
#pragma unroll
      for (int dt = 0; dt < 2; ++dt) {
        const int ro = (qa * 16 + 4 * g + (r >> 2)) * RS + dt * 16 + 4 * (r & 3);
        const s4 go = tr_read(dOs + ro), qo = tr_read(Qs + ro);
        dva[dt] = mma16<T>(go, pa_a, dva[dt]);
        dvb[dt] = mma16<T>(go, pa_b, dvb[dt]);
        dka[dt] = mma16<T>(qo, sa_a, dka[dt]);
        dkb[dt] = mma16<T>(qo, sa_b, dkb[dt]);
      }
    };
    s4 ppa = {0, 0, 0, 0}, spa = ppa, ppb = ppa, spb = ppa;   // an even query tile's P / dS waiting for its pair
#pragma unroll
    for (int qt = 0; qt < NTR; ++qt)
      if (qt < NT) {
        s4 pa, sa, pb, sb;
        tile(qt, dqacc[qt], pa, sa, pb, sb);
        if (qt & 1) dvdk2(qt - 1, ppa, spa, ppb, spb, qt, pa, sa, pb, sb);
        else { ppa = pa; spa = sa; ppb = pb; spb = sb; }
      }
    if (NT & 1) dvdk1(NT - 1, ppa, spa, ppb, spb);
    // dK, dV of both tiles: lane holds [d = dt*16 + 4g + i][key]
#pragma unroll
    for (int t2 = 0; t2 < 2; ++t2) {
      const int kk = t2 ? kb : ka;
      if (kk >= kvalid) continue;
      const int64_t krow = (kvrow0 + kb0 + kk) * HD + h * kD;
#pragma unroll
      for (int dt = 0; dt < 2; ++dt) {
        const f4 kk4 = (t2 ? dkb[dt] : dka[dt]) * scale;
        const f4 vv4 = t2 ? dvb[dt] : dva[dt];
        *reinterpret_cast<s4*>(dk + krow + dt * 16 + 4 * g) = pack4<T>(kk4[0], kk4[1], kk4[2], kk4[3]);
        *reinterpret_cast<s4*>(dv + krow + dt * 16 + 4 * g) = pack4<T>(vv4[0], vv4[1], vv4[2], vv4[3]);
      }
    }
  }
  // sum the four waves' register dQ^T into dqa (over the K / V images: zeroed once every wave is past its last
  // block), one wave at a time
  __syncthreads();
  for (int idx = threadIdx.x; idx < Lqp * kDQ / 4; idx += 256) reinterpret_cast<f4*>(dqa)[idx] = f4{0.f, 0.f, 0.f, 0.f};
  for (int ww = 0; ww < 4; ++ww) {
    __syncthreads();
    if (w == ww) {
#pragma unroll
      for (int qt = 0; qt < NTR; ++qt) {
        if (qt < NT) {
#pragma unroll
          for (int dt = 0; dt < 2; ++dt)
#pragma unroll
            for (int i = 0; i < 4; ++i) dqa[(qt * 16 + r) * kDQ + dt * 16 + 4 * g + i] += dqacc[qt][dt][i];
        }
      }
    }
  }
  __syncthreads();
  const int BH = gridDim.x;
  for (int idx = threadIdx.x; idx < Lq * kD; idx += 256) {
    const int qi = idx / kD, d = idx % kD;
    const float val = dqa[qi * kDQ + d] * scale;
    if (nchunks == 1)
      dq[(static_cast<int64_t>(b) * Lq + qi) * HD + h * kD + d] = Elt<T>::from_f(val);
    else
      ws_dq[((static_cast<int64_t>(c) * BH + bh) * Lq + qi) * kD + d] = val;
  }
}

size_t bwd2_lds_bytes(int Lqp, int elt) {
  size_t bytes = static_cast<size_t>(2 * Lqp + 512) * kDP * elt;   // Q, dO and two 128-row K / V images
  bytes = (bytes + 15) & ~size_t(15);
  return bytes + sizeof(float) * 2 * Lqp + sizeof(uint32_t) * 8 * Lqp + sizeof(float) * 4 * 2 * 16 * 20;
}

template <typename T>
__global__ void __launch_bounds__(256) mattn_dq_reduce_kernel(const float* __restrict__ ws_dq, int nchunks, int BH,
                                                              int H, int Lq, T* __restrict__ dq) {
  const int64_t idx = blockIdx.x * static_cast<int64_t>(blockDim.x) + threadIdx.x;
  const int64_t total = static_cast<int64_t>(BH) * Lq * kD;
  if (idx >= total) return;
  float acc = 0.f;
#pragma unroll 8
  for (int c = 0; c < nchunks; ++c) acc += ws_dq[static_cast<int64_t>(c) * total + idx];   // in chunk order
  const int d = static_cast<int>(idx % kD);
  const int64_t row = idx / kD;
  const int bh = static_cast<int>(row / Lq), qi = static_cast<int>(row % Lq);
  const int b = bh / H, h = bh % H;
  dq[(static_cast<int64_t>(b) * Lq + qi) * (H * kD) + h * kD + d] = Elt<T>::from_f(acc);
}

// ----------------------------------------------------------------------------------------------
// host
// ----------------------------------------------------------------------------------------------
// Key chunks per (b, head): aim for >= ~1024 workgroups, but no chunk shorter than minblk key blocks (each
// workgroup stages its queries and writes a partial once: short chunks are all prologue and epilogue).
int plan_chunks(int B, int H, int Lk, int* chunk_len, int* nchunks, int minblk = 2, int target = 1024) {
  const int BH = B * H;
  const int nblocks = (Lk + 63) / 64;
  int per = (nblocks * BH + target - 1) / target;
  per = per < minblk ? minblk : per;
  if (per > nblocks) per = nblocks;
  *chunk_len = per * 64;
  *nchunks = (Lk + *chunk_len - 1) / *chunk_len;
  return 0;
}
int fwd_minblk() { return std::max(1, m2f::option(m2f::kOptMattnFwdMinblk, 2)); }
// forward workgroup target: 512 when there are few (b, head) pairs -- config 4 (B = 2, Q = 200) at Lk = 16,384
// 0.065 -> 0.050 ms with half the chunks; config 2's 128 pairs keep 1024 (512 cost it 0.117 -> 0.126 ms,
// profiles/r04_v_mattn_target.txt)
int fwd_target(int B, int H) { return B * H < 64 ? 512 : 1024; }
// backward: 4 key blocks per chunk at least (every chunk re-stages Q, dO, LSE, delta and writes a dQ partial): at
// config 2 / Lk = 1,024 0.143 -> 0.063 ms, config 4 / Lk = 4,096 0.124 -> 0.068 ms, equal at Lk = 16,384
// (profiles/r04_o_mattn_minblk.txt)
int bwd_minblk() { return std::max(1, m2f::option(m2f::kOptMattnBwdMinblk, 4)); }

size_t bwd_lds_bytes(int Lqp, bool k16, int elt, int dq_copies = 1) {
  const int RS = k16 ? kDP : kD + 1;
  size_t bytes = static_cast<size_t>(2 * Lqp + 128) * RS * elt;
  bytes = (bytes + 15) & ~size_t(15);
  bytes += sizeof(float) * (2 * Lqp) + sizeof(uint32_t) * 2 * Lqp + sizeof(float) * 4 * 16 * 17 +
           sizeof(float) * (dq_copies == 1 ? Lqp * kDQ : Lqp * kD * dq_copies);
  return bytes;
}

template <typename T>
int attn_mask_impl(const char* fn, const void* logits, int B, int Q, int F, int Hin, int Win, int Hout, int Wout,
                   int row_fix, uint32_t* bits, int nwords, hipStream_t st) {
  if (!logits || !bits) return m2f::fail(M2F_EINVAL, "%s: null pointer", fn);
  if (B <= 0 || Q <= 0 || F <= 0 || Hin <= 0 || Win <= 0 || Hout <= 0 || Wout <= 0)
    return m2f::fail(M2F_EINVAL, "%s: non-positive size", fn);
  const int need = (F * Hout * Wout + 31) / 32;
  if (nwords < need) return m2f::fail(M2F_EINVAL, "%s: nwords %d < %d", fn, nwords, need);
  const size_t lds = static_cast<size_t>(nwords) * 4;
  if (lds > 60 * 1024) return m2f::fail(M2F_EUNSUPPORTED, "%s: target %dx%d too large", fn, Hout, Wout);
  attn_mask_bits_kernel<T><<<static_cast<unsigned>(B) * Q, 256, lds, st>>>(
      static_cast<const T*>(logits), F, Hin, Win, Hout, Wout, nwords, row_fix, bits);
  return m2f::check_launch(fn);
}

// mattn_block's head-per-XCD grouping where it is a bijection (option mattn_xcd = 0: the plain mapping)
int xcd_map(int B, int nch) { return m2f::option(m2f::kOptMattnXcd, 1) != 0 && (B * nch) % 8 == 0 ? 1 : 0; }

template <typename T>
int mattn_fwd_impl(const char* fn, const void* q, const void* k, const void* v, const uint32_t* bits, int B, int Lq,
                   int Lk, int H, int D, int qs, int kvs, int nw, float scale, void* out, float* lse2, float* ws,
                   size_t ws_bytes, hipStream_t st) {
  if (!q || !k || !v || !bits || !out || !lse2) return m2f::fail(M2F_EINVAL, "%s: null pointer", fn);
  if (D != kD) return m2f::fail(M2F_EUNSUPPORTED, "%s: head dim %d (only %d)", fn, D, kD);
  if (B <= 0 || Lq <= 0 || Lk <= 0 || H <= 0) return m2f::fail(M2F_EINVAL, "%s: non-positive size", fn);
  if (Lq > 512) return m2f::fail(M2F_EUNSUPPORTED, "%s: %d queries (max 512)", fn, Lq);
  if (nw < (Lk + 31) / 32) return m2f::fail(M2F_EINVAL, "%s: mask words %d < %d", fn, nw, (Lk + 31) / 32);
  // the kernel takes the block max on the unscaled scores
  if (!(scale > 0.f) || !std::isfinite(scale)) return m2f::fail(M2F_EINVAL, "%s: scale %g (need finite > 0)", fn, scale);
  const int vec = Elt<T>::k16 ? 8 : 4;
  if (qs % 4 || kvs % vec || !m2f::aligned(q, 8) || !m2f::aligned(k, 16) || !m2f::aligned(v, 16) ||
      !m2f::aligned(out, 16))
    return m2f::fail(M2F_EINVAL, "%s: misaligned operand or stride", fn);
  int chunk, nch;
  plan_chunks(B, H, Lk, &chunk, &nch, fwd_minblk(), fwd_target(B, H));
  const size_t need = nch > 1 ? sizeof(float) * static_cast<size_t>(nch) * B * H * Lq * (kD + 2) : 0;
  if (ws_bytes < need || (need && !ws)) return m2f::fail(M2F_EINVAL, "%s: workspace %zu < %zu", fn, ws_bytes, need);
  float* ws_o = ws;
  float* ws_ml = ws ? ws + static_cast<size_t>(nch) * B * H * Lq * kD : nullptr;
  const float sl2 = scale * kLog2e;
  const dim3 grid(B * H, nch);
  const int xm = xcd_map(B, nch);
  const int tiles = (Lq + 15) / 16, tpw = (tiles + 3) / 4;
  const T* qq = static_cast<const T*>(q);
  const T* kk = static_cast<const T*>(k);
  const T* vv = static_cast<const T*>(v);
  T* oo = static_cast<T*>(out);
  if (tpw <= 1)
    mattn_fwd_kernel<T, 1><<<grid, 256, 0, st>>>(qq, kk, vv, bits, Lq, Lk, H, qs, kvs, nw, sl2, chunk, oo, lse2, ws_o, ws_ml, xm);
  else if (tpw <= 2)
    mattn_fwd_kernel<T, 2><<<grid, 256, 0, st>>>(qq, kk, vv, bits, Lq, Lk, H, qs, kvs, nw, sl2, chunk, oo, lse2, ws_o, ws_ml, xm);
  else if (tpw <= 4)
    mattn_fwd_kernel<T, 4><<<grid, 256, 0, st>>>(qq, kk, vv, bits, Lq, Lk, H, qs, kvs, nw, sl2, chunk, oo, lse2, ws_o, ws_ml, xm);
  else
    mattn_fwd_kernel<T, 8><<<grid, 256, 0, st>>>(qq, kk, vv, bits, Lq, Lk, H, qs, kvs, nw, sl2, chunk, oo, lse2, ws_o, ws_ml, xm);
  int rc = m2f::check_launch(fn);
  if (rc || nch == 1) return rc;
  // option mattn_combine: 0 = one thread per (row, 4 channels), 1 = one wave per row; default: the wave form from 16
  // chunks up or when the thread form would fill fewer than 256 workgroups (config 4, B = 2: 15.4 -> 5.9 us at 32
  // chunks, 5.1 -> 4.2 us at 8; config 2's 12,800 rows x 8 chunks stay on the thread form, 5.6 vs 7.5 us;
  // profiles/r05_al_mattn_combine_ab.txt)
  const int64_t rows = static_cast<int64_t>(B) * H * Lq;
  const int cmb = m2f::option(m2f::kOptMattnCombine, -1);
  if (cmb == 1 || (cmb != 0 && (nch >= 16 || rows * (kD / 4) < 256 * 256))) {
    mattn_combine_wave_kernel<T><<<m2f::ceil_div(rows, 4), 256, 0, st>>>(ws_o, ws_ml, nch, B * H, H, Lq, oo, lse2);
  } else {
    const int64_t total = rows * (kD / 4);
    mattn_combine_kernel<T><<<m2f::ceil_div(total, 256), 256, 0, st>>>(ws_o, ws_ml, nch, B * H, H, Lq, oo, lse2);
  }
  return m2f::check_launch(fn);
}

template <typename T>
int mattn_bwd_impl(const char* fn, const void* q, const void* k, const void* v, const uint32_t* bits,
                   const void* out, const void* dout, const float* lse2, int B, int Lq, int Lk, int H, int D, int qs,
                   int kvs, int nw, float scale, void* dq, void* dk, void* dv, float* ws, size_t ws_bytes,
                   hipStream_t st) {
  if (!q || !k || !v || !bits || !out || !dout || !lse2 || !dq || !dk || !dv)
    return m2f::fail(M2F_EINVAL, "%s: null pointer", fn);
  if (D != kD) return m2f::fail(M2F_EUNSUPPORTED, "%s: head dim %d (only %d)", fn, D, kD);
  if (B <= 0 || Lq <= 0 || Lk <= 0 || H <= 0) return m2f::fail(M2F_EINVAL, "%s: non-positive size", fn);
  if (Lq > 512) return m2f::fail(M2F_EUNSUPPORTED, "%s: %d queries (max 512)", fn, Lq);
  if (nw < (Lk + 31) / 32) return m2f::fail(M2F_EINVAL, "%s: mask words %d < %d", fn, nw, (Lk + 31) / 32);
  const int vec = Elt<T>::k16 ? 8 : 4;
  if (qs % 4 || kvs % vec || !m2f::aligned(k, 16) || !m2f::aligned(v, 16) || !m2f::aligned(dk, 16) ||
      !m2f::aligned(dv, 16))
    return m2f::fail(M2F_EINVAL, "%s: misaligned operand or stride", fn);
  int chunk, nch;
  plan_chunks(B, H, Lk, &chunk, &nch, bwd_minblk());
  const size_t need = nch > 1 ? sizeof(float) * static_cast<size_t>(nch) * B * H * Lq * kD : 0;
  if (ws_bytes < need || (need && !ws)) return m2f::fail(M2F_EINVAL, "%s: workspace %zu < %zu", fn, ws_bytes, need);
  const int Lqp = (Lq + 15) / 16 * 16;
  // register dQ accumulation up to 128 queries (the decoders' Q = 100 case), per-wave LDS copies while four
  // of them fit (config 4's Q = 200), else LDS atomics; option mattn_dq_atomic = 1 forces the atomics
  const bool reg_dq = m2f::option(m2f::kOptMattnDqAtomic, 0) != 1;
  const size_t lds_wave = bwd_lds_bytes(Lqp, Elt<T>::k16, sizeof(T), 4);
  // registers up to 208 queries (config 4's Q = 200 takes 13 tiles: two waves per SIMD, where the four per-wave LDS
  // copies of mode 2 hold 106 KB and leave one wave per SIMD); mattn_dq_atomic = 2 forces the per-wave copies
  const int dqopt = m2f::option(m2f::kOptMattnDqAtomic, 0);
  const int mode = !reg_dq ? 0 : Lqp <= 128 ? 1 : (Lqp <= 208 && dqopt != 2) ? 3 : lds_wave <= 160 * 1024 ? 2 : 0;
  const size_t lds = mode == 2 ? lds_wave : bwd_lds_bytes(Lqp, Elt<T>::k16, sizeof(T));
  if (lds > 160 * 1024) return m2f::fail(M2F_EUNSUPPORTED, "%s: %zu B of LDS", fn, lds);
  // 16-bit operands with dQ in registers (Lq <= 128): two key tiles per wave (option mattn_bwd_keys = 16: one)
  if constexpr (Elt<T>::k16) {
    if (mode == 1 && m2f::option(m2f::kOptMattnBwdKeys, 32) == 32) {
      const size_t lds2 = bwd2_lds_bytes(Lqp, sizeof(T));
      if (int rc = m2f::set_max_lds(reinterpret_cast<const void*>(&mattn_bwd2_kernel<T, 8>), 160 * 1024, fn)) return rc;
      mattn_bwd2_kernel<T, 8><<<dim3(B * H, nch), 256, lds2, st>>>(
          static_cast<const T*>(q), static_cast<const T*>(k), static_cast<const T*>(v), bits,
          static_cast<const T*>(out), static_cast<const T*>(dout), lse2, Lq, Lk, H, qs, kvs, nw, scale * kLog2e, scale,
          chunk, Lqp, static_cast<T*>(dq), static_cast<T*>(dk), static_cast<T*>(dv), ws, xcd_map(B, nch));
      int rc = m2f::check_launch(fn);
      if (rc || nch == 1) return rc;
      const int64_t total = static_cast<int64_t>(B) * H * Lq * kD;
      mattn_dq_reduce_kernel<T><<<m2f::ceil_div(total, 256), 256, 0, st>>>(ws, nch, B * H, H, Lq, static_cast<T*>(dq));
      return m2f::check_launch(fn);
    }
  }
  auto kern = mode == 1   ? &mattn_bwd_kernel<T, 8>
              : mode == 3 ? &mattn_bwd_kernel<T, 13>
              : mode == 2 ? &mattn_bwd_kernel<T, -1>
                          : &mattn_bwd_kernel<T, 0>;
  if (int rc = m2f::set_max_lds(reinterpret_cast<const void*>(kern), 160 * 1024, fn)) return rc;
  const dim3 grid(B * H, nch);
  kern<<<grid, 256, lds, st>>>(
      static_cast<const T*>(q), static_cast<const T*>(k), static_cast<const T*>(v), bits, static_cast<const T*>(out),
      static_cast<const T*>(dout), lse2, Lq, Lk, H, qs, kvs, nw, scale * kLog2e, scale, chunk, Lqp,
      static_cast<T*>(dq), static_cast<T*>(dk), static_cast<T*>(dv), ws, xcd_map(B, nch));
  int rc = m2f::check_launch(fn);
  if (rc || nch == 1) return rc;
  const int64_t total = static_cast<int64_t>(B) * H * Lq * kD;
  mattn_dq_reduce_kernel<T><<<m2f::ceil_div(total, 256), 256, 0, st>>>(ws, nch, B * H, H, Lq, static_cast<T*>(dq));
  return m2f::check_launch(fn);
}

}  // namespace

// ------------------------------------------------------------------------------------------------
// C ABI
// ------------------------------------------------------------------------------------------------
extern "C" int m2f_attn_mask_bits(const void* logits, int dtype, int batch, int num_queries, int frames, int in_h,
                                  int in_w, int out_h, int out_w, int row_fix, uint32_t* bits, int nwords,
                                  void* stream) {
  hipStream_t st = static_cast<hipStream_t>(stream);
  const char* fn = "m2f_attn_mask_bits";
  switch (dtype) {
    case M2F_F32: return attn_mask_impl<float>(fn, logits, batch, num_queries, frames, in_h, in_w, out_h, out_w, row_fix, bits, nwords, st);
    case M2F_BF16: return attn_mask_impl<__bf16>(fn, logits, batch, num_queries, frames, in_h, in_w, out_h, out_w, row_fix, bits, nwords, st);
    case M2F_F16: return attn_mask_impl<_Float16>(fn, logits, batch, num_queries, frames, in_h, in_w, out_h, out_w, row_fix, bits, nwords, st);
    default: return m2f::fail(M2F_EUNSUPPORTED, "m2f_attn_mask_bits: dtype %d", dtype);
  }
}

extern "C" int m2f_masked_attn_plan(int batch, int num_queries, int num_keys, int num_heads, int* chunk_len,
                                    int* num_chunks, int64_t* fwd_workspace_bytes, int64_t* bwd_workspace_bytes) {
  int cl, nc, clb, ncb;
  plan_chunks(batch, num_heads, num_keys, &cl, &nc, fwd_minblk(), fwd_target(batch, num_heads));
  plan_chunks(batch, num_heads, num_keys, &clb, &ncb, bwd_minblk());
  if (chunk_len) *chunk_len = cl;
  if (num_chunks) *num_chunks = nc;
  const int64_t rows = static_cast<int64_t>(batch) * num_heads * num_queries;
  if (fwd_workspace_bytes) *fwd_workspace_bytes = nc > 1 ? nc * rows * (kD + 2) * 4 : 0;
  if (bwd_workspace_bytes) *bwd_workspace_bytes = ncb > 1 ? ncb * rows * kD * 4 : 0;
  return m2f::ok();
}

extern "C" int m2f_masked_attn_fwd(int dtype, const void* q, const void* k, const void* v, const uint32_t* bits,
                                   int batch, int num_queries, int num_keys, int num_heads, int head_dim,
                                   int q_row_stride, int kv_row_stride, int mask_words, float scale, void* out,
                                   float* lse, void* workspace, int64_t workspace_bytes, void* stream) {
  hipStream_t st = static_cast<hipStream_t>(stream);
  float* ws = static_cast<float*>(workspace);
  const size_t wb = workspace_bytes > 0 ? static_cast<size_t>(workspace_bytes) : 0;
  const char* fn = "m2f_masked_attn_fwd";
  switch (dtype) {
    case M2F_F32: return mattn_fwd_impl<float>(fn, q, k, v, bits, batch, num_queries, num_keys, num_heads, head_dim, q_row_stride, kv_row_stride, mask_words, scale, out, lse, ws, wb, st);
    case M2F_BF16: return mattn_fwd_impl<__bf16>(fn, q, k, v, bits, batch, num_queries, num_keys, num_heads, head_dim, q_row_stride, kv_row_stride, mask_words, scale, out, lse, ws, wb, st);
    case M2F_F16: return mattn_fwd_impl<_Float16>(fn, q, k, v, bits, batch, num_queries, num_keys, num_heads, head_dim, q_row_stride, kv_row_stride, mask_words, scale, out, lse, ws, wb, st);
    default: return m2f::fail(M2F_EUNSUPPORTED, "%s: dtype %d", fn, dtype);
  }
}

extern "C" int m2f_masked_attn_bwd(int dtype, const void* q, const void* k, const void* v, const uint32_t* bits,
                                   const void* out, const void* grad_out, const float* lse, int batch,
                                   int num_queries, int num_keys, int num_heads, int head_dim, int q_row_stride,
                                   int kv_row_stride, int mask_words, float scale, void* grad_q, void* grad_k,
                                   void* grad_v, void* workspace, int64_t workspace_bytes, void* stream) {
  hipStream_t st = static_cast<hipStream_t>(stream);
  float* ws = static_cast<float*>(workspace);
  const size_t wb = workspace_bytes > 0 ? static_cast<size_t>(workspace_bytes) : 0;
  const char* fn = "m2f_masked_attn_bwd";
  switch (dtype) {
    case M2F_F32: return mattn_bwd_impl<float>(fn, q, k, v, bits, out, grad_out, lse, batch, num_queries, num_keys, num_heads, head_dim, q_row_stride, kv_row_stride, mask_words, scale, grad_q, grad_k, grad_v, ws, wb, st);
    case M2F_BF16: return mattn_bwd_impl<__bf16>(fn, q, k, v, bits, out, grad_out, lse, batch, num_queries, num_keys, num_heads, head_dim, q_row_stride, kv_row_stride, mask_words, scale, grad_q, grad_k, grad_v, ws, wb, st);
    case M2F_F16: return mattn_bwd_impl<_Float16>(fn, q, k, v, bits, out, grad_out, lse, batch, num_queries, num_keys, num_heads, head_dim, q_row_stride, kv_row_stride, mask_words, scale, grad_q, grad_k, grad_v, ws, wb, st);
    default: return m2f::fail(M2F_EUNSUPPORTED, "%s: dtype %d", fn, dtype);
  }
}
