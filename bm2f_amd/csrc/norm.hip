// Residual add + LayerNorm over the last dimension, fp32: y = LN(a + b) * gamma + beta.
//
// The pixel decoder's encoder layer applies it twice per layer on (N*S, 256) rows
// (msdeformattn.py:92-131: norm1(src + dropout1(src2)), norm2(src + dropout3(ffn(src))); dropout is
// 0.0 in every shipped config).  It is HBM-bound: forward reads a, b and writes y (12 B/element),
// backward reads dy, a, b and writes dx (16 B/element) -- x = a + b is recomputed rather than saved.
//
// Layout: one wave per row, each lane owning NV float4 columns (C <= 256 * NV); the wave reduces its
// row with xor-shuffles.  Mean and variance are two-pass over the registers (exact centring, no
// Welford).  The backward's dgamma/dbeta column sums are kept per lane across the workgroup's
// grid-strided rows, summed over the 4 waves in LDS, written as one partial row per workgroup and
// reduced by a second pass in a fixed order (deterministic).
#include "bm2f.h"
#include "common.h"

#include <hip/hip_runtime.h>

#include <cmath>

namespace {

using f4 = float __attribute__((ext_vector_type(4)));

constexpr int kThreads = 256;
constexpr int kWaves = kThreads / 64;
constexpr int kBwdBlocksMax = 1024;

__device__ __forceinline__ float wave_sum(float v) {
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) v += __shfl_xor(v, off, 64);
  return v;
}

template <int NV>
__global__ void __launch_bounds__(kThreads) add_ln_fwd_kernel(const float* __restrict__ a, const float* __restrict__ b,
                                                            const float* __restrict__ gamma,
                                                            const float* __restrict__ beta, int64_t rows, int C,
                                                            float eps, float* __restrict__ y, float* __restrict__ mean,
                                                            float* __restrict__ rstd) {
  const int lane = threadIdx.x & 63;
  const int64_t wave0 = static_cast<int64_t>(blockIdx.x) * kWaves + (threadIdx.x >> 6);
  const int64_t nwaves = static_cast<int64_t>(gridDim.x) * kWaves;
  const int C4 = C >> 2;
  const float invC = 1.f / static_cast<float>(C);
  f4 g[NV], bt[NV];
#pragma unroll
  for (int j = 0; j < NV; ++j) {
    const int c4 = lane + 64 * j;
    g[j] = c4 < C4 ? reinterpret_cast<const f4*>(gamma)[c4] : f4{0.f, 0.f, 0.f, 0.f};
    bt[j] = c4 < C4 ? reinterpret_cast<const f4*>(beta)[c4] : f4{0.f, 0.f, 0.f, 0.f};
  }
  for (int64_t row = wave0; row < rows; row += nwaves) {
    const f4* ar = reinterpret_cast<const f4*>(a + row * C);
    const f4* br = b ? reinterpret_cast<const f4*>(b + row * C) : nullptr;
    f4 x[NV];
    float s = 0.f;
#pragma unroll
    for (int j = 0; j < NV; ++j) {
      const int c4 = lane + 64 * j;
      x[j] = f4{0.f, 0.f, 0.f, 0.f};
      if (c4 < C4) {
        x[j] = __builtin_nontemporal_load(ar + c4);
        if (br) x[j] += __builtin_nontemporal_load(br + c4);
      }
      s += (x[j][0] + x[j][1]) + (x[j][2] + x[j][3]);
    }
    const float mu = wave_sum(s) * invC;
    float v = 0.f;
#pragma unroll
    for (int j = 0; j < NV; ++j) {
      if (lane + 64 * j < C4) {
        const f4 d = x[j] - mu;
        v += (d[0] * d[0] + d[1] * d[1]) + (d[2] * d[2] + d[3] * d[3]);
      }
    }
    const float rs = rsqrtf(wave_sum(v) * invC + eps);
    f4* yr = reinterpret_cast<f4*>(y + row * C);
#pragma unroll
    for (int j = 0; j < NV; ++j) {
      const int c4 = lane + 64 * j;
      if (c4 < C4) yr[c4] = (x[j] - mu) * rs * g[j] + bt[j];
    }
    if (lane == 0) {
      mean[row] = mu;
      rstd[row] = rs;
    }
  }
}

template <int NV>
__global__ void __launch_bounds__(kThreads) add_ln_bwd_kernel(const float* __restrict__ dy, const float* __restrict__ a,
                                                            const float* __restrict__ b,
                                                            const float* __restrict__ gamma,
                                                            const float* __restrict__ mean,
                                                            const float* __restrict__ rstd, int64_t rows, int C,
                                                            float* __restrict__ dx, float* __restrict__ part) {
  __shared__ f4 red[kWaves][2][NV * 64];
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int64_t nwaves = static_cast<int64_t>(gridDim.x) * kWaves;
  const int C4 = C >> 2;
  const float invC = 1.f / static_cast<float>(C);
  f4 g[NV], dg[NV], db[NV];
#pragma unroll
  for (int j = 0; j < NV; ++j) {
    const int c4 = lane + 64 * j;
    g[j] = c4 < C4 ? reinterpret_cast<const f4*>(gamma)[c4] : f4{0.f, 0.f, 0.f, 0.f};
    dg[j] = db[j] = f4{0.f, 0.f, 0.f, 0.f};
  }
  for (int64_t row = static_cast<int64_t>(blockIdx.x) * kWaves + w; row < rows; row += nwaves) {
    const f4* ar = reinterpret_cast<const f4*>(a + row * C);
    const f4* br = b ? reinterpret_cast<const f4*>(b + row * C) : nullptr;
    const f4* gr = reinterpret_cast<const f4*>(dy + row * C);
    const float mu = mean[row], rs = rstd[row];
    f4 xh[NV], gy[NV];
    float s1 = 0.f, s2 = 0.f;
#pragma unroll
    for (int j = 0; j < NV; ++j) {
      const int c4 = lane + 64 * j;
      xh[j] = gy[j] = f4{0.f, 0.f, 0.f, 0.f};
      if (c4 < C4) {
        f4 x = __builtin_nontemporal_load(ar + c4);
        if (br) x += __builtin_nontemporal_load(br + c4);
        const f4 d = __builtin_nontemporal_load(gr + c4);
        xh[j] = (x - mu) * rs;
        dg[j] += d * xh[j];
        db[j] += d;
        gy[j] = d * g[j];
        s1 += (gy[j][0] + gy[j][1]) + (gy[j][2] + gy[j][3]);
        const f4 t = gy[j] * xh[j];
        s2 += (t[0] + t[1]) + (t[2] + t[3]);
      }
    }
    const float c1 = wave_sum(s1) * invC, c2 = wave_sum(s2) * invC;
    f4* dr = reinterpret_cast<f4*>(dx + row * C);
#pragma unroll
    for (int j = 0; j < NV; ++j) {
      const int c4 = lane + 64 * j;
      if (c4 < C4) dr[c4] = (gy[j] - c1 - xh[j] * c2) * rs;
    }
  }
  // workgroup partial of dgamma / dbeta: part[block][0][C], part[block][1][C]
#pragma unroll
  for (int j = 0; j < NV; ++j) {
    red[w][0][lane + 64 * j] = dg[j];
    red[w][1][lane + 64 * j] = db[j];
  }
  __syncthreads();
  for (int idx = threadIdx.x; idx < 2 * C4; idx += kThreads) {
    const int which = idx / C4, c4 = idx % C4;
    f4 acc = red[0][which][c4];
#pragma unroll
    for (int ww = 1; ww < kWaves; ++ww) acc += red[ww][which][c4];
    reinterpret_cast<f4*>(part + (static_cast<int64_t>(blockIdx.x) * 2 + which) * C)[c4] = acc;
  }
}

// dgamma / dbeta = column sums of the per-workgroup partials.  Block = 64 columns x 4 row phases; each
// thread walks a quarter of the partial rows with independent loads in flight, then the 4 phases are
// combined in LDS in a fixed order.
__global__ void __launch_bounds__(256) ln_param_reduce_kernel(const float* __restrict__ part, int nblocks, int C,
                                                              float* __restrict__ dgamma, float* __restrict__ dbeta) {
  __shared__ float red[4][64];
  const int col = blockIdx.x * 64 + (threadIdx.x & 63);  // over 2*C: [dgamma | dbeta]
  const int ph = threadIdx.x >> 6;
  const bool ok = col < 2 * C;
  const int which = ok ? col / C : 0, c = ok ? col % C : 0;
  float acc[4] = {0.f, 0.f, 0.f, 0.f};
  if (ok) {
    const float* p = part + static_cast<int64_t>(which) * C + c;
    int k = ph;
    for (; k + 12 < nblocks; k += 16) {
#pragma unroll
      for (int u = 0; u < 4; ++u) acc[u] += p[static_cast<int64_t>(k + 4 * u) * 2 * C];
    }
    for (; k < nblocks; k += 4) acc[0] += p[static_cast<int64_t>(k) * 2 * C];
  }
  red[ph][threadIdx.x & 63] = (acc[0] + acc[1]) + (acc[2] + acc[3]);
  __syncthreads();
  if (ph == 0 && ok) {
    const float v = (red[0][threadIdx.x] + red[1][threadIdx.x]) + (red[2][threadIdx.x] + red[3][threadIdx.x]);
    if (which == 0) {
      if (dgamma) dgamma[c] = v;
    } else if (dbeta) {
      dbeta[c] = v;
    }
  }
}

int check_args(const char* fn, int64_t rows, int C) {
  if (rows < 0 || C <= 0) return m2f::fail(M2F_EINVAL, "%s: rows %lld, C %d", fn, static_cast<long long>(rows), C);
  if (C % 4 || C > 1024) return m2f::fail(M2F_EUNSUPPORTED, "%s: C %d (need C %% 4 == 0, C <= 1024)", fn, C);
  return M2F_OK;
}

int bwd_blocks(int64_t rows) {
  const int64_t want = (rows + 16 * kWaves - 1) / (16 * kWaves);  // >= 16 rows per wave
  return static_cast<int>(want < 1 ? 1 : (want > kBwdBlocksMax ? kBwdBlocksMax : want));
}

}  // namespace

extern "C" int m2f_add_layernorm_workspace(int64_t rows, int C, int64_t* workspace_bytes) {
  if (int rc = check_args("m2f_add_layernorm_workspace", rows, C)) return rc;
  if (workspace_bytes) *workspace_bytes = static_cast<int64_t>(bwd_blocks(rows)) * 2 * C * sizeof(float);
  return m2f::ok();
}

extern "C" int m2f_add_layernorm_fwd_f32(const float* a, const float* b, const float* gamma, const float* beta,
                                         int64_t rows, int C, float eps, float* y, float* mean, float* rstd,
                                         void* stream) {
  const char* fn = "m2f_add_layernorm_fwd_f32";
  if (int rc = check_args(fn, rows, C)) return rc;
  if (!a || !gamma || !beta || !y || !mean || !rstd) return m2f::fail(M2F_EINVAL, "%s: null pointer", fn);
  if (!m2f::aligned(a, 16) || (b && !m2f::aligned(b, 16)) || !m2f::aligned(y, 16) || !m2f::aligned(gamma, 16) ||
      !m2f::aligned(beta, 16))
    return m2f::fail(M2F_EINVAL, "%s: operands must be 16-byte aligned", fn);
  if (rows == 0) return m2f::ok();
  hipStream_t st = static_cast<hipStream_t>(stream);
  const int64_t want = (rows + kWaves - 1) / kWaves;
  const int grid = static_cast<int>(want < 256 * 64 ? want : 256 * 64);
  const int nv = (C / 4 + 63) / 64;
  switch (nv) {
    case 1: add_ln_fwd_kernel<1><<<grid, kThreads, 0, st>>>(a, b, gamma, beta, rows, C, eps, y, mean, rstd); break;
    case 2: add_ln_fwd_kernel<2><<<grid, kThreads, 0, st>>>(a, b, gamma, beta, rows, C, eps, y, mean, rstd); break;
    case 3: add_ln_fwd_kernel<3><<<grid, kThreads, 0, st>>>(a, b, gamma, beta, rows, C, eps, y, mean, rstd); break;
    default: add_ln_fwd_kernel<4><<<grid, kThreads, 0, st>>>(a, b, gamma, beta, rows, C, eps, y, mean, rstd); break;
  }
  return m2f::check_launch(fn);
}

extern "C" int m2f_add_layernorm_bwd_f32(const float* grad_y, const float* a, const float* b, const float* gamma,
                                         const float* mean, const float* rstd, int64_t rows, int C, float* grad_x,
                                         float* grad_gamma, float* grad_beta, void* workspace,
                                         int64_t workspace_bytes, void* stream) {
  const char* fn = "m2f_add_layernorm_bwd_f32";
  if (int rc = check_args(fn, rows, C)) return rc;
  if (!grad_y || !a || !gamma || !mean || !rstd || !grad_x) return m2f::fail(M2F_EINVAL, "%s: null pointer", fn);
  if (!m2f::aligned(grad_y, 16) || !m2f::aligned(a, 16) || (b && !m2f::aligned(b, 16)) ||
      !m2f::aligned(grad_x, 16) || !m2f::aligned(gamma, 16))
    return m2f::fail(M2F_EINVAL, "%s: operands must be 16-byte aligned", fn);
  hipStream_t st = static_cast<hipStream_t>(stream);
  const int nblocks = bwd_blocks(rows);
  const int64_t need = static_cast<int64_t>(nblocks) * 2 * C * sizeof(float);
  if (!workspace || workspace_bytes < need)
    return m2f::fail(M2F_EINVAL, "%s: workspace %lld < %lld", fn, static_cast<long long>(workspace_bytes),
                     static_cast<long long>(need));
  float* part = static_cast<float*>(workspace);
  if (rows == 0) {
    if (grad_gamma) (void)m2f::zero_async(grad_gamma, C * sizeof(float), st);
    if (grad_beta) (void)m2f::zero_async(grad_beta, C * sizeof(float), st);
    return m2f::check_launch(fn);
  }
  const int nv = (C / 4 + 63) / 64;
  switch (nv) {
    case 1: add_ln_bwd_kernel<1><<<nblocks, kThreads, 0, st>>>(grad_y, a, b, gamma, mean, rstd, rows, C, grad_x, part); break;
    case 2: add_ln_bwd_kernel<2><<<nblocks, kThreads, 0, st>>>(grad_y, a, b, gamma, mean, rstd, rows, C, grad_x, part); break;
    case 3: add_ln_bwd_kernel<3><<<nblocks, kThreads, 0, st>>>(grad_y, a, b, gamma, mean, rstd, rows, C, grad_x, part); break;
    default: add_ln_bwd_kernel<4><<<nblocks, kThreads, 0, st>>>(grad_y, a, b, gamma, mean, rstd, rows, C, grad_x, part); break;
  }
  if (int rc = m2f::check_launch(fn)) return rc;
  if (grad_gamma || grad_beta) {
    ln_param_reduce_kernel<<<m2f::ceil_div(2 * C, 64), 256, 0, st>>>(part, nblocks, C, grad_gamma, grad_beta);
    return m2f::check_launch(fn);
  }
  return m2f::ok();
}
