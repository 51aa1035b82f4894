// Device helpers of the x3 (three-way split-bf16, fp32-accurate) MFMA kernels: gemm_x3.hip, conv_x3.hip.
#pragma once

#include <hip/hip_runtime.h>
#include <cstdint>

namespace m2f_x3 {

using f4 = float __attribute__((ext_vector_type(4)));
using f16v = float __attribute__((ext_vector_type(16)));
using bf8 = __bf16 __attribute__((ext_vector_type(8)));
using bf4 = __bf16 __attribute__((ext_vector_type(4)));

constexpr int kBK = 16;  // k per stage = one 32x32x16 MFMA step

// A/B experiment hook (tools/build_variant.py ... -DM2F_X3_SB): keep a pipeline step's prefetch loads ahead of its
// MFMAs (the scheduler otherwise sinks them behind the chunk's MFMAs, so the next step waits on them)
#ifdef M2F_X3_SB
#define M2F_X3_PREFETCH_FENCE() __builtin_amdgcn_sched_barrier(0)
#else
#define M2F_X3_PREFETCH_FENCE()
#endif

__device__ __forceinline__ f16v mfma(bf8 a, bf8 b, f16v c) {
  return __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, b, c, 0, 0, 0);
}

// the six product terms of order <= 2^-16 of (ah + am + al) . (bh + bm + bl), small terms first
__device__ __forceinline__ f16v mfma_x3(const bf8 (&a)[3], bf8 bh, bf8 bm, bf8 bl, f16v c) {
  c = mfma(a[2], bh, c);  // al.bh
  c = mfma(a[1], bm, c);  // am.bm
  c = mfma(a[0], bl, c);  // ah.bl
  c = mfma(a[1], bh, c);  // am.bh
  c = mfma(a[0], bm, c);  // ah.bm
  return mfma(a[0], bh, c);  // ah.bh
}

// bijective XCD-aware remap: consecutive logical ids land on the same XCD (blocks id, id+8, ... share one)
__device__ __forceinline__ int xcd_remap(int id, int nwg) {
  const int q = nwg / 8, r = nwg % 8, xcd = id % 8;
  return (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + id / 8;
}

// grouped XCD remap: blocks are dealt to XCDs round-robin (b % 8), so consecutive block ids cover one group
// of 8*G logical tiles at a time (the chip streams one contiguous region, spread over all HBM channels) and
// XCD b % 8 gets the contiguous run of G tiles inside it (neighbouring tiles share one L2).  Bijective:
// the partial last group keeps identity order.
__device__ __forceinline__ int xcd_group_remap(int b, int nwg, int G) {
  const int span = 8 * G, group = b / span, within = b - group * span;
  if ((group + 1) * span > nwg) return b;
  return group * span + (within & 7) * G + (within >> 3);
}

// x -> (h, m, l) exactly (x = h + m + l to the last fp32 bit); non-finite x keeps h = x, m = l = 0
__device__ __forceinline__ void split3(float x, __bf16& h, __bf16& m, __bf16& l) {
  h = static_cast<__bf16>(x);
  const float r1 = x - static_cast<float>(h);
  m = static_cast<__bf16>(r1);
  const float r2 = r1 - static_cast<float>(m);
  l = static_cast<__bf16>(r2);
  if (!isfinite(x)) { m = static_cast<__bf16>(0.f); l = static_cast<__bf16>(0.f); }
}

// split3 of 8 consecutive values into the three bf8 planes of an MFMA operand, a pair of values per
// v_cvt_pk_bf16_f32 and back-conversions by shifts / masks of the packed word: 15 VALU per pair, no
// branches (so the compiler can interleave it with the MFMAs of the previous chunk).  Non-finite x: the
// remainder x - h is NaN exactly then, and is replaced by 0 (h = x, m = l = 0, as split3).
__device__ __forceinline__ void split8(const float (&x)[8], bf8 (&fa)[3]) {
  using u4 = unsigned __attribute__((ext_vector_type(4)));
  using b2 = __bf16 __attribute__((ext_vector_type(2)));
  u4 h, m, l;
#pragma unroll
  for (int p = 0; p < 4; ++p) {
    const float x0 = x[2 * p], x1 = x[2 * p + 1];
    const unsigned hp = __builtin_bit_cast(unsigned, b2{static_cast<__bf16>(x0), static_cast<__bf16>(x1)});
    float r0 = x0 - __uint_as_float(hp << 16), r1 = x1 - __uint_as_float(hp & 0xffff0000u);
    r0 = r0 == r0 ? r0 : 0.f;
    r1 = r1 == r1 ? r1 : 0.f;
    const unsigned mp = __builtin_bit_cast(unsigned, b2{static_cast<__bf16>(r0), static_cast<__bf16>(r1)});
    const float s0 = r0 - __uint_as_float(mp << 16), s1 = r1 - __uint_as_float(mp & 0xffff0000u);
    const unsigned lp = __builtin_bit_cast(unsigned, b2{static_cast<__bf16>(s0), static_cast<__bf16>(s1)});
    h[p] = hp;
    m[p] = mp;
    l[p] = lp;
  }
  fa[0] = __builtin_bit_cast(bf8, h);
  fa[1] = __builtin_bit_cast(bf8, m);
  fa[2] = __builtin_bit_cast(bf8, l);
}

// B images are rows of 16 bf16 (32 B) with the two 16-B halves swapped on rows whose bit 3 is set: the
// dense image is then conflict-free for the 32x32x16 operand read (ds_read_b128 lane groups
// {0-3,12-15,20-27}, ... cover all 64 banks once)
__device__ __forceinline__ int swz(int n) { return (n >> 3) & 1; }

}  // namespace m2f_x3
