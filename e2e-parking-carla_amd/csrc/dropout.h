// Counter-based dropout masks shared by the attention, feed-forward and LayerNorm kernels:
// keep(c) = (mix(c ^ seedmix) >> 8) / 2^24 >= p for element counter c, seedmix derived from a
// per-call device seed.  Regenerated in the backward, so no mask is ever stored.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace e2ep {

__device__ __forceinline__ uint32_t att_mix(uint32_t x) {  // 32-bit integer finaliser
  x ^= x >> 16;
  x *= 0x7feb352du;
  x ^= x >> 15;
  x *= 0x846ca68bu;
  x ^= x >> 16;
  return x;
}
// dropout keep test for counter c: uniform 24-bit value >= p
__device__ __forceinline__ bool att_keep(uint32_t seedmix, uint32_t c, float p) {
  return (float)(att_mix(c ^ seedmix) >> 8) * (1.0f / 16777216.0f) >= p;
}
__device__ __forceinline__ uint32_t att_seedmix(const int *seed) {
  return seed ? att_mix((uint32_t)seed[0] * 0x9e3779b9u + 0x632be5abu) : 0u;
}

}  // namespace e2ep
