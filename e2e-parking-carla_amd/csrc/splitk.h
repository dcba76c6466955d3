// In-kernel split-K reduction ("the last block of a tile reduces").
//
// A GEMM whose K range is split over gridDim.z blocks per output tile used to write raw
// partial slabs and leave the sum to a second, separate reduction launch.  In the HIP-graph
// replayed train step that second launch costs ~5 us of kernel time plus the inter-kernel
// gap, ~200 times per step.  Instead every block of a split tile stores its partial slab,
// then increments the tile's arrival counter; the block that arrives last (whichever split
// it is) reads all the tile's slabs IN SPLIT ORDER — the same fixed-order sum as the former
// reduction kernel, so results stay bitwise deterministic — applies the epilogue, writes the
// final values and resets the counter to 0 for the next launch.  No block ever waits for
// another (no spinning, no co-residency assumption).
//
// Counters: each translation unit that uses this declares one pool of device counters
// (zero at load, E2EP_TILE_POOL) and hands every launch its own range of it (tile_range):
// round robin, so launches that may run concurrently (graph replays, side streams) never
// share counters, and every counter is 0 again once its launch has finished.
#pragma once
#include <mutex>

#include "common.h"

namespace e2ep {

constexpr unsigned TILE_POOL = 1u << 18;  // counters per pool (1 MiB)

#define E2EP_TILE_POOL(name) static __device__ unsigned name[e2ep::TILE_POOL]

// Host side: first counter of a fresh range of n (<= TILE_POOL) counters of a pool whose
// allocation cursor is `next`.
inline unsigned tile_range(unsigned &next, unsigned n) {
  static std::mutex mu;
  std::lock_guard<std::mutex> lock(mu);
  if (next + n > TILE_POOL) next = 0;
  const unsigned base = next;
  next += n;
  return base;
}

// Device address of a pool (resolved once per pool).
template <typename T>
inline unsigned *pool_ptr(const T &symbol, unsigned *&cache) {
  if (!cache) {
    void *p = nullptr;
    if (hipGetSymbolAddress(&p, symbol) == hipSuccess) cache = static_cast<unsigned *>(p);
  }
  return cache;
}

// Partial slabs are written and read with system-coherent buffer accesses (cache policy sc0
// sc1: stores write through every cache level, loads miss them), so neither an L2 writeback
// (an agent-scope release fence writes back the whole XCD L2 — ~100 us over a ~900-block
// split grid) nor an L2 invalidate is needed: waiting for this thread's stores to complete
// orders them before the arrival increment.
constexpr int CPOL_SYS = 1 | 16;  // sc0 | sc1
__device__ __forceinline__ void store_sys(__amdgpu_buffer_rsrc_t r, int byte_off, float v) {
  __builtin_amdgcn_raw_buffer_store_b32(__builtin_bit_cast(unsigned, v), r, byte_off, 0, CPOL_SYS);
}
__device__ __forceinline__ float load_sys(__amdgpu_buffer_rsrc_t r, int byte_off) {
  return __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(r, byte_off, 0, CPOL_SYS));
}

// Every thread of the block calls this after storing its partial slab with store_sys.
// Returns true, in all threads, in the block that arrived last at `counter` out of `splits`;
// that block may then read the other blocks' slabs with load_sys.
__device__ __forceinline__ bool splitk_last(unsigned *counter, int splits) {
  __shared__ unsigned s_prev;
  __builtin_amdgcn_s_waitcnt(0);  // this thread's write-through stores have completed
  __syncthreads();
  if (threadIdx.x == 0)
    s_prev = __hip_atomic_fetch_add(counter, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  __syncthreads();
  const bool last = s_prev == (unsigned)(splits - 1);
  if (last && threadIdx.x == 0)
    __hip_atomic_exchange(counter, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  return last;
}

}  // namespace e2ep
