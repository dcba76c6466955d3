// In-launch hand-offs between workgroups (gfx950: per-XCD L2s are not coherent with each
// other; cdna_hip_programming.md §6 Guideline 16, MI355X_MICROARCH.md § visibility).
//
// Form used here (the visibility table's first row): every byte handed to another workgroup
// is stored write-through (sc1), every storing wave drains its stores (s_waitcnt vmcnt(0)),
// the workgroup meets at a barrier, then ONE lane adds to an agent-scope arrival counter; the
// workgroup whose add returns the last ticket reads the handed-off bytes with sc1 loads only
// (no acquire fence, no plain load of them).  The last arriver also resets its counter, so a
// counter slot is zero again when the launch ends.
//
// Counters come from one zero-initialised device pool per device (handoff.hip): each launch
// takes a fresh slot range from a host-side cursor, so kernels that may run concurrently
// (side-stream weight gradients, several captured graphs) never share a slot; a captured
// launch keeps its range on every replay (kernels of one graph replay never overlap
// themselves).  Launches captured into a graph take their ranges from a region that is
// handed out once (HANDOFF_CAPTURED counters, never reused while the process lives; once they
// run out, ~500 captured train steps, later captures get none and use separate reduce
// launches); eager launches rotate through the other region, so an eager launch never shares
// a slot with a live graph's launch.
#pragma once
#include "common.h"

namespace e2ep {

constexpr int HANDOFF_POOL = 1 << 24;      // counters in a device's pool (64 MB)
constexpr int HANDOFF_CAPTURED = 15 << 20; // of them for launches captured into graphs

// n zeroed counters for one launch on `stream` (host; the current device's pool), or nullptr
// when n is out of range or the pool cannot be fetched: the callers then run their split-K
// reductions as separate launches
unsigned int *handoff_slots(int n, hipStream_t stream);

__device__ __forceinline__ void st_sc1(float *p, float v) {
  __hip_atomic_store(reinterpret_cast<unsigned int *>(p), __builtin_bit_cast(unsigned int, v),
                     __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ float ld_sc1(const float *p) {
  return __builtin_bit_cast(float, __hip_atomic_load(reinterpret_cast<const unsigned int *>(p),
                                                     __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT));
}

__device__ __forceinline__ void st_sc1_d(double *p, double v) {
  __hip_atomic_store(reinterpret_cast<unsigned long long *>(p),
                     __builtin_bit_cast(unsigned long long, v), __ATOMIC_RELAXED,
                     __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ double ld_sc1_d(const double *p) {
  return __builtin_bit_cast(double, __hip_atomic_load(reinterpret_cast<const unsigned long long *>(p),
                                                      __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT));
}

// 16-B write-through store / sc1 load through a buffer descriptor (aux 16 = sc1).  The LLVM
// intrinsics are bound directly, as bload4 in common.h.
__device__ void e2ep_raw_buffer_store_v4f32(e2ep_f4 v, __amdgpu_buffer_rsrc_t rsrc, int voffset,
                                            int soffset, int aux) __asm("llvm.amdgcn.raw.ptr.buffer.store.v4f32");
__device__ __forceinline__ void bstore4_sc1(__amdgpu_buffer_rsrc_t r, int byte_off, float4 v) {
  e2ep_f4 w;
  w[0] = v.x; w[1] = v.y; w[2] = v.z; w[3] = v.w;
  e2ep_raw_buffer_store_v4f32(w, r, byte_off, 0, 16);
}
__device__ __forceinline__ float4 bload4_sc1(__amdgpu_buffer_rsrc_t r, int byte_off) {
  const e2ep_f4 v = e2ep_raw_buffer_load_v4f32(r, byte_off, 0, 16);
  return make_float4(v[0], v[1], v[2], v[3]);
}
__device__ __forceinline__ void bstore_sc1(__amdgpu_buffer_rsrc_t r, int byte_off, float v) {
  __builtin_amdgcn_raw_buffer_store_b32(__builtin_bit_cast(unsigned, v), r, byte_off, 0, 16);
}
__device__ __forceinline__ float bload_sc1(__amdgpu_buffer_rsrc_t r, int byte_off) {
  return __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(r, byte_off, 0, 16));
}

// Every storing wave: drain this wave's write-through stores.
__device__ __forceinline__ void handoff_drain() { asm volatile("s_waitcnt vmcnt(0)" ::: "memory"); }

// After handoff_drain() in every wave: barrier, one arrival on *cnt, returns (to every thread
// of the workgroup) whether this workgroup arrived last of `arrivals`; the last one resets
// the counter.  `flag` is a __shared__ int of the caller.
__device__ __forceinline__ bool handoff_arrive(unsigned int *cnt, unsigned int arrivals, int *flag) {
  __syncthreads();
  if (threadIdx.x == 0) {
    const unsigned int old = __hip_atomic_fetch_add(cnt, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    const bool last = old == arrivals - 1;
    if (last) __hip_atomic_store(cnt, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    *flag = last;
  }
  __syncthreads();
  return *flag != 0;
}

}  // namespace e2ep
