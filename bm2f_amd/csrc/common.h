// Shared helpers for the libbm2f C ABI: per-thread error strings and launch checking.
#pragma once

#include <hip/hip_runtime.h>
#include <cstdarg>
#include <cstdint>
#include <cstdio>
#include <string>

#include "bm2f.h"

namespace m2f {

std::string& last_error();

inline int fail(int code, const char* fmt, ...) {
  char buf[512];
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(buf, sizeof(buf), fmt, ap);
  va_end(ap);
  last_error() = buf;
  return code;
}

inline int ok() {
  last_error().clear();
  return M2F_OK;
}

// Check the launch that was just issued on this thread (hipGetLastError clears the sticky state).
inline int check_launch(const char* what) {
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) return fail(M2F_ELAUNCH, "%s: %s", what, hipGetErrorString(e));
  return ok();
}

inline bool aligned(const void* p, size_t a) { return (reinterpret_cast<uintptr_t>(p) % a) == 0; }

inline unsigned ceil_div(int64_t a, int64_t b) { return static_cast<unsigned>((a + b - 1) / b); }

// Explicit tuning options (m2f_set_option, include/bm2f.h): geometry and engine overrides for tests and
// tools.  The library never reads the environment; an unset option means the built-in default.  Every
// option changes the partition or the kernel variant only, never the arithmetic's result.
enum Option : int {
  kOptMsdaThreads, kOptMsdaTile, kOptMsdaTileW, kOptMsdaHalo, kOptMsdaWinRows, kOptMsdaBwdTiled, kOptMsdaFwdTiled,
  kOptMattnDqAtomic, kOptGemmNtCfg, kOptX3TnNw, kOptX3TnBlocks, kOptX3NtCfg, kOptMsdaFwdQuad, kOptMsdaBwdOverlap, kOptMsdaBwdDet, kOptMsdaFwdPb, kOptMsdaBwdRatio,
  kOptMsdaFwdLds, kOptMsdaFwdTile, kOptMsdaFwdTileW, kOptMsdaFwdCap, kOptMsdaFwdHalo,
  kOptMattnFwdMinblk, kOptMattnBwdMinblk, kOptMaskDfStage, kOptMattnBwdKeys, kOptMattnXcd, kOptMattnCombine, kOptMsdaBwdRowSort, kOptMsdaBwdWalk4, kOptMsdaFwdXcd, kOptMsdaFwdPair, kOptCount
};
int64_t option_raw(Option o);  // -1 when unset

// Zero `bytes` bytes at p on stream st with a kernel, not hipMemsetAsync: on this ROCm a memset captured in a HIP
// graph is not re-run correctly when the graph is replayed (tools/graph_memset_check.py), and callers capture the
// library's launches in graphs (bench_model.GraphStep).  Returns a HIP error code.
hipError_t zero_async(void* p, size_t bytes, hipStream_t st);
// The same for a rows x cols fp32 matrix at row stride ld floats (a kernel: no memset node in a captured graph).
hipError_t zero2d_f32_async(float* p, int64_t ld, int64_t cols, int64_t rows, hipStream_t st);
// Raise `kernel`'s dynamic-LDS limit to `bytes` on the current device, once per (kernel, device, bytes) and
// thread-safe; returns M2F_OK or an M2F_ELAUNCH status (with the HIP error in last_error) naming `fn`.
int set_max_lds(const void* kernel, int bytes, const char* fn);
inline int option(Option o, int dflt) {
  const int64_t v = option_raw(o);
  return v < 0 ? dflt : static_cast<int>(v);
}

}  // namespace m2f
