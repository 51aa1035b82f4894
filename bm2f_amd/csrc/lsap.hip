// Batched linear sum assignment (Hungarian matching) on the GPU.
//
// The reference matches every decoder head's predictions to the targets with scipy's
// linear_sum_assignment on the host, one image at a time (mask2former/modeling/matcher.py:309-311:
// C.cpu() then LSAP), i.e. a device->host sync per image per head.  Here one wavefront solves one
// problem: the shortest-augmenting-path algorithm scipy implements (Crouse 2016, a Jonker-Volgenant
// variant), in fp64 on the fp32 costs, with the per-row Dijkstra scan over the columns spread over the
// 64 lanes and the column choice reduced with scipy's tie rule (lowest reduced cost; among equal ones an
// unassigned column, the last one in scan order; else the first).  Problems are (rows <= 256) x
// (cols <= 1024) after orienting them so rows <= cols, as scipy does (it transposes a tall matrix).
//
// Output per problem: match[r] = the column matched to original row r, or -1 -- for a tall cost matrix
// (queries x targets) every target gets exactly one query.
#include "bm2f.h"
#include "common.h"

#include <hip/hip_runtime.h>

#include <cfloat>

namespace {

constexpr int kMaxRows = 256;   // the smaller side (targets per image)
constexpr int kMaxCols = 1024;  // the larger side (queries)

// one wave per problem; cost(r, c) of the oriented problem = C[trans ? c : r][trans ? r : c]
__global__ void __launch_bounds__(64) lsap_kernel(const float* __restrict__ C, int64_t batch_stride, int ld,
                                                  const int* __restrict__ nrows_orig, int ncols_orig_max,
                                                  const int* __restrict__ ncols_orig, int* __restrict__ match,
                                                  int64_t match_stride, int* __restrict__ status) {
  __shared__ double u[kMaxRows], v[kMaxCols], spc[kMaxCols];
  __shared__ int path[kMaxCols], row4col[kMaxCols], col4row[kMaxRows], remaining[kMaxCols];
  __shared__ unsigned char SR[kMaxRows], SC[kMaxCols];
  const int b = blockIdx.x, lane = threadIdx.x;
  const int R0 = nrows_orig[b], C0 = ncols_orig ? ncols_orig[b] : ncols_orig_max;
  const bool trans = R0 > C0;
  const int nr = trans ? C0 : R0, nc = trans ? R0 : C0;
  const float* Cb = C + b * batch_stride;
  int* mb = match + b * match_stride;
  for (int i = lane; i < R0; i += 64) mb[i] = -1;
  if (nr == 0) {
    if (lane == 0) status[b] = 0;
    return;
  }
  if (nr > kMaxRows || nc > kMaxCols) {
    if (lane == 0) status[b] = 2;
    return;
  }
  auto cost = [&](int r, int c) -> double {
    return static_cast<double>(trans ? Cb[static_cast<int64_t>(c) * ld + r] : Cb[static_cast<int64_t>(r) * ld + c]);
  };
  // scipy rejects NaN and -inf entries up front ("matrix contains invalid numeric entries")
  bool bad = false;
  for (int e = lane; e < nr * nc; e += 64) {
    const double c = cost(e / nc, e % nc);
    bad |= (c != c) || c == -HUGE_VAL;
  }
  if (__any(bad)) {
    if (lane == 0) status[b] = 3;
    return;
  }
  for (int i = lane; i < nr; i += 64) { u[i] = 0.0; col4row[i] = -1; }
  for (int j = lane; j < nc; j += 64) { v[j] = 0.0; row4col[j] = -1; }
  __syncthreads();
  bool ok = true;
  for (int cur = 0; cur < nr && ok; ++cur) {
    // ---- augmenting path from row cur --------------------------------------------------------------
    double minv = 0.0;
    int nrem = nc;
    for (int it = lane; it < nc; it += 64) { remaining[it] = nc - it - 1; spc[it] = DBL_MAX; path[it] = -1; SC[it] = 0; }
    for (int i = lane; i < nr; i += 64) SR[i] = 0;
    __syncthreads();
    int sink = -1, i = cur;
    while (sink == -1) {
      if (lane == 0) SR[i] = 1;
      // each lane scans remaining[it] for it = lane, lane + 64, ...: first its own best under scipy's rule
      double best = DBL_MAX;
      int bidx = -1;
      bool bun = false;  // best is an unassigned column
      for (int it = lane; it < nrem; it += 64) {
        const int j = remaining[it];
        const double r = minv + cost(i, j) - u[i] - v[j];
        if (r < spc[j]) { path[j] = i; spc[j] = r; }
        const double s = spc[j];
        const bool un = row4col[j] == -1;
        if (s < best || (s == best && un)) { best = s; bidx = it; bun = un; }
      }
      // combine lanes in scan order: ties resolve as the sequential scan would (a later unassigned column
      // wins a tie, an assigned one never displaces an equal earlier choice)
      for (int off = 1; off < 64; off <<= 1) {
        const double ob = __shfl_xor(best, off);
        const int oi = __shfl_xor(bidx, off);
        const bool ou = __shfl_xor(static_cast<int>(bun), off) != 0;
        // the candidate that comes later in scan order "wins" a tie only if it is unassigned
        const bool other_later = oi > bidx;
        bool take;
        if (oi < 0) take = false;
        else if (bidx < 0) take = true;
        else if (ob < best) take = true;
        else if (ob > best) take = false;
        else take = other_later ? ou : !bun;  // equal: a later unassigned wins; an earlier one wins unless we are unassigned
        if (take) { best = ob; bidx = oi; bun = ou; }
      }
      __syncthreads();
      minv = best;
      if (bidx < 0 || best >= DBL_MAX) { ok = false; break; }  // infeasible (inf / nan costs)
      const int j = remaining[bidx];
      if (row4col[j] == -1) sink = j;
      else i = row4col[j];
      __syncthreads();
      if (lane == 0) {
        SC[j] = 1;
        remaining[bidx] = remaining[nrem - 1];
      }
      --nrem;
      __syncthreads();
    }
    if (!ok) break;
    // ---- dual update and augmentation ---------------------------------------------------------------
    if (lane == 0) u[cur] += minv;
    for (int r = lane; r < nr; r += 64)
      if (SR[r] && r != cur) u[r] += minv - spc[col4row[r]];
    for (int c = lane; c < nc; c += 64)
      if (SC[c]) v[c] -= minv - spc[c];
    __syncthreads();
    if (lane == 0) {
      int j = sink;
      while (true) {
        const int r = path[j];
        row4col[j] = r;
        const int t = col4row[r];
        col4row[r] = j;
        j = t;
        if (r == cur) break;
      }
    }
    __syncthreads();
  }
  if (!ok) {
    if (lane == 0) status[b] = 1;
    return;
  }
  // original orientation: row r of C (a query when trans) <- column
  if (trans) {
    for (int c = lane; c < nc; c += 64)
      if (row4col[c] >= 0) mb[c] = row4col[c];
  } else {
    for (int r = lane; r < nr; r += 64) mb[r] = col4row[r];
  }
  if (lane == 0) status[b] = 0;
}

}  // namespace

extern "C" int m2f_lsap_batched(const float* cost, int batch, int max_rows, int max_cols, int64_t batch_stride,
                                const int* rows, const int* cols, int* match, int* status, void* stream) {
  const char* fn = "m2f_lsap_batched";
  if (batch < 0 || max_rows < 0 || max_cols < 0 || !rows || !match || !status || (batch > 0 && !cost))
    return m2f::fail(M2F_EINVAL, "%s: bad arguments", fn);
  // per-problem size limits (min side <= kMaxRows, max side <= kMaxCols) are reported in status[b] = 2
  if (batch == 0) return m2f::ok();
  hipStream_t st = static_cast<hipStream_t>(stream);
  lsap_kernel<<<batch, 64, 0, st>>>(cost, batch_stride, max_cols, rows, max_cols, cols, match, max_rows, status);
  return m2f::check_launch(fn);
}
