// Shared helpers for the libe2ep_hip.so kernels (gfx950 only).
#pragma once
#include <hip/hip_runtime.h>
#include <stdarg.h>
#include <stdio.h>

#include "e2ep.h"

namespace e2ep {

void set_error(const char *fmt, ...);

inline hipStream_t as_stream(void *s) { return reinterpret_cast<hipStream_t>(s); }

// Launch-status check: returns the code to propagate (0 = ok).
inline int launch_status(const char *what) {
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) {
    set_error("%s: %s", what, hipGetErrorString(e));
    return (int)e;
  }
  return 0;
}

inline int cdiv(long long a, long long b) { return (int)((a + b - 1) / b); }

// 64-lane wave helpers
__device__ __forceinline__ float wave_sum(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}

}  // namespace e2ep

#define E2EP_REQUIRE(cond, code, ...)      \
  do {                                     \
    if (!(cond)) {                         \
      e2ep::set_error(__VA_ARGS__);        \
      return (code);                       \
    }                                      \
  } while (0)
