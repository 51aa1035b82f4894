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

}  // namespace m2f
