// Arrival-counter pools for the in-launch hand-offs of handoff.h.
#include <mutex>

#include "handoff.h"

namespace e2ep {

__device__ unsigned int g_handoff_pool[HANDOFF_POOL];  // zero at load; last arrivers re-zero

namespace {
constexpr int MAXDEV = 64;
struct Pool {
  unsigned int *base = nullptr;
  int captured = 0;                 // next range of the captured region [0, HANDOFF_CAPTURED)
  int eager = HANDOFF_CAPTURED;     // next range of the rotating region [HANDOFF_CAPTURED, POOL)
};
Pool g_pools[MAXDEV];
std::mutex g_mu;  // autograd's backward thread launches too
}  // namespace

unsigned int *handoff_slots(int n, hipStream_t stream) {
  if (n <= 0 || n > HANDOFF_POOL - HANDOFF_CAPTURED) return nullptr;
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess || dev < 0 || dev >= MAXDEV) return nullptr;
  hipStreamCaptureStatus cs = hipStreamCaptureStatusNone;
  const bool captured = hipStreamIsCapturing(stream, &cs) == hipSuccess &&
                        cs == hipStreamCaptureStatusActive;
  std::lock_guard<std::mutex> lock(g_mu);
  Pool &p = g_pools[dev];
  if (!p.base) {  // the device's own copy of the pool (module globals are per device)
    void *a = nullptr;
    if (hipGetSymbolAddress(&a, HIP_SYMBOL(g_handoff_pool)) != hipSuccess) return nullptr;
    p.base = static_cast<unsigned int *>(a);
  }
  const int len = (n + 63) & ~63;  // 256-B aligned ranges
  int at;
  if (captured) {
    // exhausted: no range (the caller runs its separate reduce launches).  Never wrap: the
    // oldest ranges may belong to graphs that are still alive and replay concurrently
    if (p.captured + len > HANDOFF_CAPTURED) return nullptr;
    at = p.captured;
    p.captured += len;
  } else {
    if (p.eager + len > HANDOFF_POOL) p.eager = HANDOFF_CAPTURED;
    at = p.eager;
    p.eager += len;
  }
  return p.base + at;
}

}  // namespace e2ep
