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

// bf16 activation storage (C3: the depthwise outputs and their gradients, e2ep.h E2EP_IO_*):
// typed 4-wide loads / stores whose arithmetic stays fp32 — a bf16 tensor element is widened
// on load and rounded to nearest-even (v_cvt_pk_bf16_f32) on store.
typedef __bf16 bf16_t;
typedef __bf16 e2ep_bf16x4 __attribute__((ext_vector_type(4)));
__device__ __forceinline__ float4 ld4(const float *p) { return *reinterpret_cast<const float4 *>(p); }
__device__ __forceinline__ float4 ld4(const bf16_t *p) {
  const e2ep_bf16x4 h = *reinterpret_cast<const e2ep_bf16x4 *>(p);
  return make_float4((float)h[0], (float)h[1], (float)h[2], (float)h[3]);
}
__device__ __forceinline__ void st4(float *p, float4 v) { *reinterpret_cast<float4 *>(p) = v; }
__device__ __forceinline__ void st4(bf16_t *p, float4 v) {
  const e2ep_bf16x4 h = {(bf16_t)v.x, (bf16_t)v.y, (bf16_t)v.z, (bf16_t)v.w};
  *reinterpret_cast<e2ep_bf16x4 *>(p) = h;
}
__device__ __forceinline__ float ld1(const float *p) { return *p; }
__device__ __forceinline__ float ld1(const bf16_t *p) { return (float)*p; }
__device__ __forceinline__ void st1(float *p, float v) { *p = v; }
__device__ __forceinline__ void st1(bf16_t *p, float v) { *p = (bf16_t)v; }
// the value a store of v into a T tensor keeps (statistics of stored outputs)
template <typename T>
__device__ __forceinline__ float stored(float v) { return (float)(T)v; }
// 4 elements of a T tensor through a buffer descriptor (byte offset of the first element)
__device__ __forceinline__ float4 bload4t(__amdgpu_buffer_rsrc_t r, int byte_off, const float *) {
  return bload4(r, byte_off);
}
__device__ __forceinline__ float4 bload4t(__amdgpu_buffer_rsrc_t r, int byte_off, const bf16_t *) {
  const e2ep_f2 u = e2ep_raw_buffer_load_v2f32(r, byte_off, 0, 0);
  const e2ep_bf16x4 h = __builtin_bit_cast(e2ep_bf16x4, u);
  return make_float4((float)h[0], (float)h[1], (float)h[2], (float)h[3]);
}

// one element of a T tensor through a buffer descriptor (load widened, store rounded)
__device__ __forceinline__ float bload_t(__amdgpu_buffer_rsrc_t r, int byte_off, const float *) {
  return bload(r, byte_off);
}
__device__ __forceinline__ float bload_t(__amdgpu_buffer_rsrc_t r, int byte_off, const bf16_t *) {
  const unsigned short h = __builtin_amdgcn_raw_buffer_load_b16(r, byte_off, 0, 0);
  return __builtin_bit_cast(float, (unsigned)h << 16);
}
__device__ __forceinline__ void bstore_t(__amdgpu_buffer_rsrc_t r, int byte_off, float v, float *) {
  bstore(r, byte_off, v);
}
__device__ __forceinline__ void bstore_t(__amdgpu_buffer_rsrc_t r, int byte_off, float v, bf16_t *) {
  __builtin_amdgcn_raw_buffer_store_b16(__builtin_bit_cast(unsigned short, (bf16_t)v), r, byte_off, 0, 0);
}

// sigmoid(z) = 1 / (1 + e^-z) for the per-element activations (swish and its derivative in the
// BatchNorm / depthwise / squeeze-excitation kernels, the SE gate): e^-z as v_exp_f32 of
// -z log2(e) and the reciprocal as v_rcp_f32 (1 ulp) instead of the correctly rounded divide
// this library is built with (-fhip-fp32-correctly-rounded-divide-sqrt: ~10 instructions per
// divide).  Error: rounding -log2(e) * z to fp32 before v_exp_f32 perturbs e^-z by a relative
// |z| * 2^-24 (v_exp_f32 / v_rcp_f32 add a few ulp), so sigmoid_f / swish_f are within
// 2^-24 * (2 |z| + 8) relative of the exact value — measured worst 3.9e-6 (~65 ulp) at
// z = -44; where sigmoid(z) is no longer a normal fp32 number (z < -87.3) the reciprocal's
// denormal is flushed to 0, an absolute error under 2^-126.
// tests/test_nn_ops_gpu.py::test_sigmoid_swish_error_bound holds them to that bound against
// fp64 over [-90, 90].  Those kernels run one or two sigmoids per
// element and were ALU-bound on the 128² maps.  The losses keep expf (loss.hip).
__device__ __forceinline__ float sigmoid_f(float z) {
  return __builtin_amdgcn_rcpf(1.f + __builtin_amdgcn_exp2f(-1.4426950408889634f * z));
}
__device__ __forceinline__ float swish_f(float z) { return z * sigmoid_f(z); }

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
