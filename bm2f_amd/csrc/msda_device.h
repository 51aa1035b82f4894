// Device helpers shared by the MSDA kernels (msda.hip, msda_fused.hip).  Header-only, internal.
#pragma once

#include <hip/hip_runtime.h>
#include <cstdint>

namespace m2f_msda {

using f4 = float __attribute__((ext_vector_type(4)));
using f2 = float __attribute__((ext_vector_type(2)));

// ------------------------------------------------------------------------------------------------
// fp32 fast path: G = D/4 lanes per (n,q,m) pair, float4 per lane.
// ------------------------------------------------------------------------------------------------

struct Corners {
  int64_t o1, o2, o3, o4;     // element offsets of the 4 corner rows (clamped to valid rows)
  int h0, w0;                 // top-left corner (may be -1; meaningful when ok)
  float w1, w2, w3, w4;       // bilinear weights
  float hy, ly, hx, lx;       // 1-lh, lh, 1-lw, lw
  bool c1, c2, c3, c4;        // corner inside the level
  bool ok;                    // sample inside (-1,H)x(-1,W)
};

__device__ __forceinline__ Corners make_corners(float locx, float locy, int H, int W, int64_t lbase, int64_t rs) {
  Corners k;
  const float h = locy * H - 0.5f;
  const float w = locx * W - 0.5f;
  k.ok = h > -1.f && w > -1.f && h < static_cast<float>(H) && w < static_cast<float>(W);
  const float hs = k.ok ? h : -2.f, ws = k.ok ? w : -2.f;   // invalid point: every corner outside
  const float fh = floorf(hs), fw = floorf(ws);
  const int h0 = static_cast<int>(fh), w0 = static_cast<int>(fw);
  k.h0 = h0; k.w0 = w0;
  k.ly = hs - fh; k.lx = ws - fw;
  k.hy = 1.f - k.ly; k.hx = 1.f - k.lx;
  k.w1 = k.hy * k.hx; k.w2 = k.hy * k.lx; k.w3 = k.ly * k.hx; k.w4 = k.ly * k.lx;
  k.c1 = h0 >= 0 && w0 >= 0;
  k.c2 = h0 >= 0 && w0 + 1 <= W - 1;
  k.c3 = h0 + 1 <= H - 1 && w0 >= 0;
  k.c4 = h0 + 1 <= H - 1 && w0 + 1 <= W - 1;
  // clamp every corner into the level so the (masked) loads never leave it, valid point or not
  const int y0 = min(max(h0, 0), H - 1), y1 = min(max(h0 + 1, 0), H - 1);
  const int x0 = min(max(w0, 0), W - 1), x1 = min(max(w0 + 1, 0), W - 1);
  k.o1 = lbase + (static_cast<int64_t>(y0) * W + x0) * rs;
  k.o2 = lbase + (static_cast<int64_t>(y0) * W + x1) * rs;
  k.o3 = lbase + (static_cast<int64_t>(y1) * W + x0) * rs;
  k.o4 = lbase + (static_cast<int64_t>(y1) * W + x1) * rs;
  return k;
}

// make_corners with 32-bit element offsets (callers guarantee every offset < 2^31): the 64-bit multiply-adds
// of the general form are quarter-rate VALU sequences, four per sample
struct Corners32 {
  int o1, o2, o3, o4;
  float w1, w2, w3, w4;
  bool c1, c2, c3, c4;
  bool ok;
};

__device__ __forceinline__ Corners32 make_corners32(float locx, float locy, int H, int W, int lbase, int rs) {
  Corners32 k;
  const float h = locy * H - 0.5f;
  const float w = locx * W - 0.5f;
  k.ok = h > -1.f && w > -1.f && h < static_cast<float>(H) && w < static_cast<float>(W);
  const float hs = k.ok ? h : -2.f, ws = k.ok ? w : -2.f;
  const float fh = floorf(hs), fw = floorf(ws);
  const int h0 = static_cast<int>(fh), w0 = static_cast<int>(fw);
  const float ly = hs - fh, lx = ws - fw, hy = 1.f - ly, hx = 1.f - lx;
  k.w1 = hy * hx; k.w2 = hy * lx; k.w3 = ly * hx; k.w4 = ly * lx;
  k.c1 = h0 >= 0 && w0 >= 0;
  k.c2 = h0 >= 0 && w0 + 1 <= W - 1;
  k.c3 = h0 + 1 <= H - 1 && w0 >= 0;
  k.c4 = h0 + 1 <= H - 1 && w0 + 1 <= W - 1;
  const int y0 = min(max(h0, 0), H - 1), y1 = min(max(h0 + 1, 0), H - 1);
  const int x0 = min(max(w0, 0), W - 1), x1 = min(max(w0 + 1, 0), W - 1);
  // one multiply for the block: the other corners are 0 / 1 pixel right and 0 / 1 row down of corner 1
  const int dx = x1 != x0 ? rs : 0, dy = y1 != y0 ? W * rs : 0;
  k.o1 = lbase + (y0 * W + x0) * rs;
  k.o2 = k.o1 + dx;
  k.o3 = k.o1 + dy;
  k.o4 = k.o3 + dx;
  return k;
}

// x / d for the sampling-offset normalisation (ms_deform_attn.py:106-109, offset / (W, H)).  When d is a
// power of two, x * (1 / d) is the same correctly rounded value (both are exact scalings of x by 2^-k), so
// the IEEE division sequence (about ten VALU) is skipped; otherwise it is a true division.
__device__ __forceinline__ float div_norm(float x, float d, float inv, bool pow2) { return pow2 ? x * inv : x / d; }

__device__ __forceinline__ f4 ld4(const float* p) { return *reinterpret_cast<const f4*>(p); }

constexpr int kTileMaxL = 4;

struct TileGeom {
  int L;
  int H[kTileMaxL], W[kTileMaxL], start[kTileMaxL];
  int nty, ntx;   // tile grid shared by all levels
  int max_rows;   // list-head cells per workgroup (the window grid extended by one row / column)
  int max_halo;   // windows never extend more than this many pixels past the tile
  int max_qt;     // queries of the largest tile (sizes the LDS carve-up)
  float invW[kTileMaxL], invH[kTileMaxL];  // 1 / W, 1 / H (used where they are powers of two: exact)
  int ratio23;    // backward: phase-2 units per phase-3 unit at the head of the merged queue
  int rowsort;    // backward: phase-3 rows dealt in order of their record count (1) or window order (0)
  int walk4;      // backward: phase-3 records four per step, decoded once per quad (1) or two per step (0)
  int xcdmap;     // forward: block b's (tile, head) from XCD b % 8 (a contiguous tile range per XCD, all heads of a
                  // tile on one XCD) (1) or the head fastest (0)
};

__device__ __forceinline__ int tile_lo(int t, int n, int nt) { return (t * n) / nt; }

// the tile t with tile_lo(t) <= y < tile_lo(t + 1)
__device__ __forceinline__ int tile_of(int y, int n, int nt) {
  int t = (y * nt + nt - 1) / n;
  while (t > 0 && tile_lo(t, n, nt) > y) --t;
  while (t + 1 < nt && tile_lo(t + 1, n, nt) <= y) ++t;
  return t;
}

// Sum over each aligned group of 8 lanes with DPP moves (VALU, no LDS crossbar): xor 1, xor 2 within
// quads, then row_half_mirror (lane i <-> 7-i) pairs the two quads.
__device__ __forceinline__ float sum8_dpp(float v) {
  v += __builtin_bit_cast(float, __builtin_amdgcn_update_dpp(0, __builtin_bit_cast(int, v), 0xB1, 0xF, 0xF, false));
  v += __builtin_bit_cast(float, __builtin_amdgcn_update_dpp(0, __builtin_bit_cast(int, v), 0x4E, 0xF, 0xF, false));
  v += __builtin_bit_cast(float, __builtin_amdgcn_update_dpp(0, __builtin_bit_cast(int, v), 0x141, 0xF, 0xF, false));
  return v;
}

// DPP quad permutation (CTRL = quad_perm selector) of a float
template <int CTRL>
__device__ __forceinline__ float qperm(float v) {
  return __builtin_bit_cast(float, __builtin_amdgcn_update_dpp(0, __builtin_bit_cast(int, v), CTRL, 0xF, 0xF, false));
}

// max over each aligned group of 8 lanes (exact and order-free, unlike a sum)
__device__ __forceinline__ float max8_dpp(float v) {
  v = fmaxf(v, __builtin_bit_cast(float, __builtin_amdgcn_update_dpp(0, __builtin_bit_cast(int, v), 0xB1, 0xF, 0xF, false)));
  v = fmaxf(v, __builtin_bit_cast(float, __builtin_amdgcn_update_dpp(0, __builtin_bit_cast(int, v), 0x4E, 0xF, 0xF, false)));
  v = fmaxf(v, __builtin_bit_cast(float, __builtin_amdgcn_update_dpp(0, __builtin_bit_cast(int, v), 0x141, 0xF, 0xF, false)));
  return v;
}

// DPP quad_perm moves with bound_ctrl (every lane of a quad reads a lane of its own quad, so no "old" operand);
// CTRL = p * 0x55 broadcasts quad lane p, 0xB1 / 0x4E exchange with lane xor 1 / xor 2
template <int CTRL>
__device__ __forceinline__ int qpermi(int v) { return __builtin_amdgcn_mov_dpp(v, CTRL, 0xF, 0xF, true); }
template <int CTRL>
__device__ __forceinline__ float qpermf(float v) {
  return __builtin_bit_cast(float, __builtin_amdgcn_mov_dpp(__builtin_bit_cast(int, v), CTRL, 0xF, 0xF, true));
}

// 16 bytes at a 32-bit byte offset from base (global_load with an SGPR base and a 32-bit VGPR offset)
__device__ __forceinline__ f4 ldb4(const char* base, unsigned boff) {
  return *reinterpret_cast<const f4*>(base + boff);
}

// One sampling point's bilinear geometry for the quad kernels, in 32-bit BYTE offsets (value bytes < 2^31):
// corner byte offsets (rows clamped into the level, so every load stays inside it) and the four bilinear weights
// with a corner outside the level weighted 0.  (h, w) = (loc_y * H - 0.5, loc_x * W - 0.5); a point outside
// (-1, H) x (-1, W) (NaN included) is moved to (-2, -2), where every corner lies outside (weights 0, ok false).
// The clamps run on the floored floats (v_med3_f32 takes the SGPR bound; the integer form needs two ops).
// a * b + c on the 24-bit multiplier (operands < 2^24, result < 2^32): LLVM turns __umul24(a, b) + c into
// v_mad_u64_u32, a multi-pass instruction
__device__ __forceinline__ int mad_u24(int a, int b, int c) {
  int r;
  asm("v_mad_u32_u24 %0, %1, %2, %3" : "=v"(r) : "v"(a), "v"(b), "v"(c));
  return r;
}

struct QuadPoint {
  int o1, o2, o3, o4;
  float w1, w2, w3, w4;
  float ly, lx;
  bool c1, c2, c3, c4;  // corner inside the level
  bool ok;
};

__device__ __forceinline__ QuadPoint quad_point(float h, float w, int H, int W, int lbase, int rsb) {
  QuadPoint k;
  const float fHm1 = static_cast<float>(H - 1), fWm1 = static_cast<float>(W - 1);
  k.ok = h > -1.f && w > -1.f && h < static_cast<float>(H) && w < static_cast<float>(W);
  const float hs = k.ok ? h : -2.f, ws = k.ok ? w : -2.f;
  const float fh = floorf(hs), fw = floorf(ws);
  const float ly = hs - fh, lx = ws - fw, hy = 1.f - ly, hx = 1.f - lx;
  const bool vy0 = fh >= 0.f, vy1 = fh < fHm1, vx0 = fw >= 0.f, vx1 = fw < fWm1;
  const int y0 = static_cast<int>(__builtin_amdgcn_fmed3f(fh, 0.f, fHm1));
  const int x0 = static_cast<int>(__builtin_amdgcn_fmed3f(fw, 0.f, fWm1));
  k.o1 = mad_u24(mad_u24(y0, W, x0), rsb, lbase);
  const int dx = (vx0 && vx1) ? rsb : 0, dy = (vy0 && vy1) ? W * rsb : 0;
  k.o2 = k.o1 + dx;
  k.o3 = k.o1 + dy;
  k.o4 = k.o3 + dx;
  k.c1 = vy0 && vx0;
  k.c2 = vy0 && vx1;
  k.c3 = vy1 && vx0;
  k.c4 = vy1 && vx1;
  k.w1 = k.c1 ? hy * hx : 0.f;
  k.w2 = k.c2 ? hy * lx : 0.f;
  k.w3 = k.c3 ? ly * hx : 0.f;
  k.w4 = k.c4 ? ly * lx : 0.f;
  k.ly = ly;
  k.lx = lx;
  return k;
}

// quad_point from a point's floors and fractions (h = fh + ly, w = fw + lx; fh = fw = -2 and ly = lx = 0 for a point
// outside, as quad_point moves it): the same offsets, weights and flags as quad_point(h, w, ...)
__device__ __forceinline__ QuadPoint quad_point_fl(int fh, int fw, float ly, float lx, int H, int W, int lbase, int rsb) {
  QuadPoint k;
  k.ok = fh != -2;
  const float hy = 1.f - ly, hx = 1.f - lx;
  const bool vy0 = fh >= 0, vy1 = fh < H - 1, vx0 = fw >= 0, vx1 = fw < W - 1;
  const int y0 = static_cast<int>(__builtin_amdgcn_fmed3f(static_cast<float>(fh), 0.f, static_cast<float>(H - 1)));
  const int x0 = static_cast<int>(__builtin_amdgcn_fmed3f(static_cast<float>(fw), 0.f, static_cast<float>(W - 1)));
  k.o1 = mad_u24(mad_u24(y0, W, x0), rsb, lbase);
  const int dx = (vx0 && vx1) ? rsb : 0, dy = (vy0 && vy1) ? W * rsb : 0;
  k.o2 = k.o1 + dx;
  k.o3 = k.o1 + dy;
  k.o4 = k.o3 + dx;
  k.c1 = vy0 && vx0;
  k.c2 = vy0 && vx1;
  k.c3 = vy1 && vx0;
  k.c4 = vy1 && vx1;
  k.w1 = k.c1 ? hy * hx : 0.f;
  k.w2 = k.c2 ? hy * lx : 0.f;
  k.w3 = k.c3 ? ly * hx : 0.f;
  k.w4 = k.c4 ? ly * lx : 0.f;
  k.ly = ly;
  k.lx = lx;
  return k;
}

__device__ __forceinline__ float pick4(const f4& v, int c) {
  return c == 0 ? v.x : (c == 1 ? v.y : (c == 2 ? v.z : v.w));
}


}  // namespace m2f_msda
