// GroupNorm (+ ReLU), fp32 NCHW: the pixel decoder's GN layers (msdeformattn.py:216-219 input_proj,
// :269-281 adapter_1 / layer_1 via detectron2 Conv2d(norm=GN(32), activation=relu)); the reference runs
// them in fp32 (autocast off, :314,320).  torch runs statistics, the normalisation and the ReLU as three
// passes (and three more backward); here:
//   forward   gn_stats (each group is one contiguous span of C/G * HW floats: split blocks, fp64 partial
//             sums, fixed-order combine -> mean, rstd per (n, g)) and gn_apply (y = x * a + b' with
//             torch's fused a = rstd * gamma, b' = beta - mean * a, ReLU in the same pass, float4);
//   backward  gn_bwd_plane (per (n, c): ds = sum g x, db = sum g with g = dy masked by the ReLU, the mask
//             recomputed from x with the forward's exact expression), gn_bwd_coef (per (n, g): torch's
//             c2, c3), gn_bwd_apply (dx = c1 g + c2 x + c3, float4) and gn_bwd_param (dgamma, dbeta sums
//             over n in a fixed order).  Deterministic; HBM-bound (fwd 2 reads + 1 write, bwd 4 reads +
//             1 write per element).
#include "bm2f.h"
#include "common.h"

#include <hip/hip_runtime.h>

#include <cmath>

namespace {

using f4 = float __attribute__((ext_vector_type(4)));

constexpr int kT = 256;

__device__ __forceinline__ double block_sum(double v, double* red) {
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) v += __shfl_xor(v, off, 64);
  const int w = threadIdx.x >> 6, lane = threadIdx.x & 63;
  __syncthreads();
  if (lane == 0) red[w] = v;
  __syncthreads();
  double s = 0.0;
  for (int i = 0; i < kT / 64; ++i) s += red[i];
  return s;
}

// grid (N*G, splits): partial (sum, sumsq) of span [split*len/splits, ...) of group ng
__global__ void __launch_bounds__(kT) gn_stats(const float* __restrict__ x, int64_t span, int splits,
                                               double* __restrict__ part) {
  __shared__ double red[kT / 64];
  const int64_t ng = blockIdx.x;
  const int sp = blockIdx.y;
  const int64_t nv = span / 4;
  const int64_t v0 = nv * sp / splits, v1 = nv * (sp + 1) / splits;
  const f4* p = reinterpret_cast<const f4*>(x + ng * span);
  double s = 0.0, q = 0.0;
  for (int64_t i = v0 + threadIdx.x; i < v1; i += kT) {
    // squares and sums in fp64: E[x^2] - E[x]^2 cancels catastrophically for |mean| >> std if the squares
    // are rounded to fp32 first (x = randn + 100: fp32 squares carry 6e-4 absolute error each)
    const f4 v = p[i];
    const double a = v.x, b = v.y, c = v.z, d = v.w;
    s += (a + b) + (c + d);
    q += (a * a + b * b) + (c * c + d * d);
  }
  s = block_sum(s, red);
  q = block_sum(q, red);
  if (threadIdx.x == 0) {
    part[(ng * splits + sp) * 2] = s;
    part[(ng * splits + sp) * 2 + 1] = q;
  }
}

__global__ void gn_finalize(const double* __restrict__ part, int splits, int64_t ngroups, double inv_n, float eps,
                            float* __restrict__ mean, float* __restrict__ rstd) {
  const int64_t ng = blockIdx.x * static_cast<int64_t>(blockDim.x) + threadIdx.x;
  if (ng >= ngroups) return;
  double s = 0.0, q = 0.0;
  for (int i = 0; i < splits; ++i) {
    s += part[(ng * splits + i) * 2];
    q += part[(ng * splits + i) * 2 + 1];
  }
  const double m = s * inv_n;
  double var = q * inv_n - m * m;
  var = var < 0.0 ? 0.0 : var;
  mean[ng] = static_cast<float>(m);
  rstd[ng] = static_cast<float>(1.0 / sqrt(var + static_cast<double>(eps)));
}

__device__ __forceinline__ void fused_ab(const float* mean, const float* rstd, const float* gamma,
                                         const float* beta, int64_t n, int c, int C, int cpg, float& a, float& b) {
  const int64_t ng = n * (C / cpg) + c / cpg;
  const float r = rstd[ng];
  a = gamma ? r * gamma[c] : r;
  b = (beta ? beta[c] : 0.f) - mean[ng] * a;
}

template <bool RELU>
__global__ void __launch_bounds__(kT) gn_apply(const float* __restrict__ x, const float* __restrict__ mean,
                                               const float* __restrict__ rstd, const float* __restrict__ gamma,
                                               const float* __restrict__ beta, float* __restrict__ y, int C,
                                               int cpg, int hw4, int64_t nvec) {
  const int64_t i = blockIdx.x * static_cast<int64_t>(kT) + threadIdx.x;
  if (i >= nvec) return;
  const int64_t nc = i / hw4;
  const int c = static_cast<int>(nc % C);
  float a, b;
  fused_ab(mean, rstd, gamma, beta, nc / C, c, C, cpg, a, b);
  f4 v = reinterpret_cast<const f4*>(x)[i];
  v.x = fmaf(v.x, a, b); v.y = fmaf(v.y, a, b); v.z = fmaf(v.z, a, b); v.w = fmaf(v.w, a, b);
  if (RELU) { v.x = fmaxf(v.x, 0.f); v.y = fmaxf(v.y, 0.f); v.z = fmaxf(v.z, 0.f); v.w = fmaxf(v.w, 0.f); }
  reinterpret_cast<f4*>(y)[i] = v;
}

// per (n, c) plane: ds = sum g x, db = sum g, g = dy (masked where the forward output was <= 0)
template <bool RELU>
__global__ void __launch_bounds__(kT) gn_bwd_plane(const float* __restrict__ dy, const float* __restrict__ x,
                                                   const float* __restrict__ mean, const float* __restrict__ rstd,
                                                   const float* __restrict__ gamma, const float* __restrict__ beta,
                                                   int C, int cpg, int hw4, double* __restrict__ dsdb) {
  __shared__ double red[kT / 64];
  const int64_t nc = blockIdx.x;
  const int c = static_cast<int>(nc % C);
  float a = 0.f, b = 0.f;
  if (RELU) fused_ab(mean, rstd, gamma, beta, nc / C, c, C, cpg, a, b);
  const f4* xp = reinterpret_cast<const f4*>(x) + nc * hw4;
  const f4* gp = reinterpret_cast<const f4*>(dy) + nc * hw4;
  double ds = 0.0, db = 0.0;
  for (int i = threadIdx.x; i < hw4; i += kT) {
    const f4 xv = xp[i];
    f4 g = gp[i];
    if (RELU) {
      g.x = fmaf(xv.x, a, b) > 0.f ? g.x : 0.f; g.y = fmaf(xv.y, a, b) > 0.f ? g.y : 0.f;
      g.z = fmaf(xv.z, a, b) > 0.f ? g.z : 0.f; g.w = fmaf(xv.w, a, b) > 0.f ? g.w : 0.f;
    }
    ds += static_cast<double>((g.x * xv.x + g.y * xv.y) + (g.z * xv.z + g.w * xv.w));
    db += static_cast<double>((g.x + g.y) + (g.z + g.w));
  }
  ds = block_sum(ds, red);
  db = block_sum(db, red);
  if (threadIdx.x == 0) {
    dsdb[nc * 2] = ds;
    dsdb[nc * 2 + 1] = db;
  }
}

// per (n, g): torch's GroupNorm backward coefficients, dx = c1[c] g + c2 x + c3 with c1 = rstd gamma[c]
__global__ void gn_bwd_coef(const double* __restrict__ dsdb, const float* __restrict__ mean,
                            const float* __restrict__ rstd, const float* __restrict__ gamma, int C, int cpg,
                            int64_t ngroups, double inv_n, float* __restrict__ c23) {
  const int64_t ng = blockIdx.x * static_cast<int64_t>(blockDim.x) + threadIdx.x;
  if (ng >= ngroups) return;
  const int G = C / cpg;
  const int64_t n = ng / G;
  const int g0 = static_cast<int>(ng % G) * cpg;
  double sds = 0.0, sdb = 0.0;
  for (int k = 0; k < cpg; ++k) {
    const int c = g0 + k;
    const double gm = gamma ? gamma[c] : 1.0;
    sds += dsdb[(n * C + c) * 2] * gm;
    sdb += dsdb[(n * C + c) * 2 + 1] * gm;
  }
  const double m = mean[ng], r = rstd[ng];
  const double c2 = (sdb * m - sds) * r * r * r * inv_n;
  const double c3 = -c2 * m - sdb * r * inv_n;
  c23[ng * 2] = static_cast<float>(c2);
  c23[ng * 2 + 1] = static_cast<float>(c3);
}

template <bool RELU>
__global__ void __launch_bounds__(kT) gn_bwd_apply(const float* __restrict__ dy, const float* __restrict__ x,
                                                   const float* __restrict__ mean, const float* __restrict__ rstd,
                                                   const float* __restrict__ gamma, const float* __restrict__ beta,
                                                   const float* __restrict__ c23, float* __restrict__ dx, int C,
                                                   int cpg, int hw4, int64_t nvec) {
  const int64_t i = blockIdx.x * static_cast<int64_t>(kT) + threadIdx.x;
  if (i >= nvec) return;
  const int64_t nc = i / hw4;
  const int c = static_cast<int>(nc % C);
  const int64_t ng = (nc / C) * (C / cpg) + c / cpg;
  float a = 0.f, b = 0.f;
  if (RELU) fused_ab(mean, rstd, gamma, beta, nc / C, c, C, cpg, a, b);
  const float c1 = gamma ? rstd[ng] * gamma[c] : rstd[ng];
  const float c2 = c23[ng * 2], c3 = c23[ng * 2 + 1];
  const f4 xv = reinterpret_cast<const f4*>(x)[i];
  f4 g = reinterpret_cast<const f4*>(dy)[i];
  if (RELU) {
    g.x = fmaf(xv.x, a, b) > 0.f ? g.x : 0.f; g.y = fmaf(xv.y, a, b) > 0.f ? g.y : 0.f;
    g.z = fmaf(xv.z, a, b) > 0.f ? g.z : 0.f; g.w = fmaf(xv.w, a, b) > 0.f ? g.w : 0.f;
  }
  f4 o;
  o.x = c1 * g.x + c2 * xv.x + c3; o.y = c1 * g.y + c2 * xv.y + c3;
  o.z = c1 * g.z + c2 * xv.z + c3; o.w = c1 * g.w + c2 * xv.w + c3;
  reinterpret_cast<f4*>(dx)[i] = o;
}

// dgamma[c] = sum_n (ds - db mean) rstd, dbeta[c] = sum_n db (fixed order over n)
__global__ void gn_bwd_param(const double* __restrict__ dsdb, const float* __restrict__ mean,
                             const float* __restrict__ rstd, int N, int C, int cpg, float* __restrict__ dgamma,
                             float* __restrict__ dbeta) {
  const int c = blockIdx.x * blockDim.x + threadIdx.x;
  if (c >= C) return;
  const int G = C / cpg;
  double dg = 0.0, dbt = 0.0;
  for (int n = 0; n < N; ++n) {
    const int64_t ng = static_cast<int64_t>(n) * G + c / cpg;
    const int64_t k = (static_cast<int64_t>(n) * C + c) * 2;
    const double ds = dsdb[k], db = dsdb[k + 1];
    dg += (ds - db * mean[ng]) * rstd[ng];
    dbt += db;
  }
  if (dgamma) dgamma[c] = static_cast<float>(dg);
  if (dbeta) dbeta[c] = static_cast<float>(dbt);
}

int gn_check(const char* fn, int N, int C, int G, int64_t HW) {
  if (N <= 0 || C <= 0 || G <= 0 || HW <= 0 || C % G) return m2f::fail(M2F_EINVAL, "%s: bad sizes", fn);
  if (HW % 4) return m2f::fail(M2F_EUNSUPPORTED, "%s: needs H*W %% 4 == 0", fn);
  return M2F_OK;
}

int gn_splits(int64_t ngroups, int64_t span) {
  int s = static_cast<int>((2048 + ngroups - 1) / ngroups);
  const int64_t maxs = (span / 4 + 1023) / 1024;
  if (s > maxs) s = static_cast<int>(maxs);
  return s < 1 ? 1 : s;
}

}  // namespace

extern "C" int m2f_group_norm_workspace(int N, int C, int G, int64_t HW, int64_t* workspace_bytes) {
  int rc = gn_check("m2f_group_norm_workspace", N, C, G, HW);
  if (rc) return rc;
  const int64_t ng = static_cast<int64_t>(N) * G;
  const int64_t fwd = ng * gn_splits(ng, HW * (C / G)) * 16;
  const int64_t bwd = static_cast<int64_t>(N) * C * 16 + ng * 8;
  if (workspace_bytes) *workspace_bytes = (fwd > bwd ? fwd : bwd) + 256;
  return m2f::ok();
}

extern "C" int m2f_group_norm_fwd_f32(const float* x, const float* gamma, const float* beta, int N, int C, int G,
                                      int64_t HW, float eps, int relu, float* y, float* mean, float* rstd,
                                      void* workspace, int64_t workspace_bytes, void* stream) {
  const char* fn = "m2f_group_norm_fwd_f32";
  int rc = gn_check(fn, N, C, G, HW);
  if (rc) return rc;
  if (!x || !y || !mean || !rstd || !workspace) return m2f::fail(M2F_EINVAL, "%s: null pointer", fn);
  if (!m2f::aligned(x, 16) || !m2f::aligned(y, 16) || !m2f::aligned(workspace, 16))
    return m2f::fail(M2F_EINVAL, "%s: x, y, workspace must be 16-byte aligned", fn);
  const int64_t ng = static_cast<int64_t>(N) * G, span = HW * (C / G);
  const int splits = gn_splits(ng, span);
  if (workspace_bytes < ng * splits * 16) return m2f::fail(M2F_EINVAL, "%s: workspace too small", fn);
  if (ng > 0x7fffffff) return m2f::fail(M2F_EUNSUPPORTED, "%s: too many groups", fn);
  hipStream_t st = static_cast<hipStream_t>(stream);
  double* part = static_cast<double*>(workspace);
  gn_stats<<<dim3(static_cast<unsigned>(ng), splits), kT, 0, st>>>(x, span, splits, part);
  if ((rc = m2f::check_launch(fn))) return rc;
  gn_finalize<<<m2f::ceil_div(ng, 256), 256, 0, st>>>(part, splits, ng, 1.0 / static_cast<double>(span), eps, mean,
                                                      rstd);
  if ((rc = m2f::check_launch(fn))) return rc;
  const int64_t nvec = static_cast<int64_t>(N) * C * HW / 4;
  const int hw4 = static_cast<int>(HW / 4), cpg = C / G;
  if (relu)
    gn_apply<true><<<m2f::ceil_div(nvec, kT), kT, 0, st>>>(x, mean, rstd, gamma, beta, y, C, cpg, hw4, nvec);
  else
    gn_apply<false><<<m2f::ceil_div(nvec, kT), kT, 0, st>>>(x, mean, rstd, gamma, beta, y, C, cpg, hw4, nvec);
  return m2f::check_launch(fn);
}

extern "C" int m2f_group_norm_bwd_f32(const float* dy, const float* x, const float* mean, const float* rstd,
                                      const float* gamma, const float* beta, int N, int C, int G, int64_t HW,
                                      int relu, float* dx, float* dgamma, float* dbeta, void* workspace,
                                      int64_t workspace_bytes, void* stream) {
  const char* fn = "m2f_group_norm_bwd_f32";
  int rc = gn_check(fn, N, C, G, HW);
  if (rc) return rc;
  if (!dy || !x || !mean || !rstd || !dx || !workspace) return m2f::fail(M2F_EINVAL, "%s: null pointer", fn);
  if (!m2f::aligned(x, 16) || !m2f::aligned(dy, 16) || !m2f::aligned(dx, 16) || !m2f::aligned(workspace, 16))
    return m2f::fail(M2F_EINVAL, "%s: dy, x, dx, workspace must be 16-byte aligned", fn);
  const int64_t ng = static_cast<int64_t>(N) * G, nc = static_cast<int64_t>(N) * C;
  if (workspace_bytes < nc * 16 + ng * 8) return m2f::fail(M2F_EINVAL, "%s: workspace too small", fn);
  if (nc > 0x7fffffff) return m2f::fail(M2F_EUNSUPPORTED, "%s: too many planes", fn);
  hipStream_t st = static_cast<hipStream_t>(stream);
  double* dsdb = static_cast<double*>(workspace);
  float* c23 = reinterpret_cast<float*>(dsdb + nc * 2);
  const int hw4 = static_cast<int>(HW / 4), cpg = C / G;
  if (relu)
    gn_bwd_plane<true><<<static_cast<unsigned>(nc), kT, 0, st>>>(dy, x, mean, rstd, gamma, beta, C, cpg, hw4, dsdb);
  else
    gn_bwd_plane<false><<<static_cast<unsigned>(nc), kT, 0, st>>>(dy, x, mean, rstd, gamma, beta, C, cpg, hw4, dsdb);
  if ((rc = m2f::check_launch(fn))) return rc;
  const double inv_n = 1.0 / static_cast<double>(HW * cpg);
  gn_bwd_coef<<<m2f::ceil_div(ng, 256), 256, 0, st>>>(dsdb, mean, rstd, gamma, C, cpg, ng, inv_n, c23);
  if ((rc = m2f::check_launch(fn))) return rc;
  const int64_t nvec = nc * HW / 4;
  if (relu)
    gn_bwd_apply<true><<<m2f::ceil_div(nvec, kT), kT, 0, st>>>(dy, x, mean, rstd, gamma, beta, c23, dx, C, cpg, hw4,
                                                               nvec);
  else
    gn_bwd_apply<false><<<m2f::ceil_div(nvec, kT), kT, 0, st>>>(dy, x, mean, rstd, gamma, beta, c23, dx, C, cpg, hw4,
                                                                nvec);
  if ((rc = m2f::check_launch(fn))) return rc;
  if (dgamma || dbeta) {
    gn_bwd_param<<<m2f::ceil_div(C, 256), 256, 0, st>>>(dsdb, mean, rstd, N, C, cpg, dgamma, dbeta);
    return m2f::check_launch(fn);
  }
  return m2f::ok();
}
