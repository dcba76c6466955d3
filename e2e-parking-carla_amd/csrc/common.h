// Shared helpers for the libe2ep_hip.so kernels (gfx950 only).
#pragma once
#include <hip/hip_runtime.h>
#include <stdarg.h>
#include <stdio.h>

#include "e2ep.h"
#include "tune.h"

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

// Branch-free guarded memory access.  `if (ok) v = p[i];` inside an unrolled loop makes
// hipcc branch around every load and wait vmcnt(0) per element, serialising the loads; a
// buffer load with an out-of-range byte offset instead returns 0 (a store is dropped), so
// the guard becomes a select.  Descriptors must be built from wave-uniform values.
constexpr int OOR = 0x7ffffff0;
__device__ __forceinline__ __amdgpu_buffer_rsrc_t rsrc(const void *p, long long bytes) {
  const int nr = bytes >= 0x7fffffff ? 0x7fffffff : (int)bytes;
  return __builtin_amdgcn_make_buffer_rsrc(const_cast<void *>(p), (short)0, nr, 0x00020000);
}
__device__ __forceinline__ float bload(__amdgpu_buffer_rsrc_t r, int byte_off) {
  return __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(r, byte_off, 0, 0));
}
__device__ __forceinline__ int bload_i(__amdgpu_buffer_rsrc_t r, int byte_off) {
  return (int)__builtin_amdgcn_raw_buffer_load_b32(r, byte_off, 0, 0);
}
// 16-B buffer load.  (__builtin_amdgcn_raw_buffer_load_b128 is lowered to a single dword
// load by the ROCm 7.2 compiler, so the LLVM intrinsic is bound directly.)
typedef float e2ep_f4 __attribute__((ext_vector_type(4)));
__device__ e2ep_f4 e2ep_raw_buffer_load_v4f32(__amdgpu_buffer_rsrc_t rsrc, int voffset, int soffset,
                                              int aux) __asm("llvm.amdgcn.raw.ptr.buffer.load.v4f32");
__device__ __forceinline__ float4 bload4(__amdgpu_buffer_rsrc_t r, int byte_off) {
  const e2ep_f4 v = e2ep_raw_buffer_load_v4f32(r, byte_off, 0, 0);
  return make_float4(v[0], v[1], v[2], v[3]);
}
// 8-B buffer load (same binding as bload4)
typedef float e2ep_f2 __attribute__((ext_vector_type(2)));
__device__ e2ep_f2 e2ep_raw_buffer_load_v2f32(__amdgpu_buffer_rsrc_t rsrc, int voffset, int soffset,
                                              int aux) __asm("llvm.amdgcn.raw.ptr.buffer.load.v2f32");
__device__ __forceinline__ float2 bload2(__amdgpu_buffer_rsrc_t r, int byte_off) {
  const e2ep_f2 v = e2ep_raw_buffer_load_v2f32(r, byte_off, 0, 0);
  return make_float2(v[0], v[1]);
}
__device__ __forceinline__ void bstore(__amdgpu_buffer_rsrc_t r, int byte_off, float v) {
  __builtin_amdgcn_raw_buffer_store_b32(__builtin_bit_cast(unsigned, v), r, byte_off, 0, 0);
}

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
