// Arrival-counter pool for the in-launch hand-offs of handoff.h.
#include <mutex>

#include "handoff.h"

namespace e2ep {

__device__ unsigned int g_handoff_pool[HANDOFF_POOL];  // zero at load; last arrivers re-zero

unsigned int *handoff_slots(int n) {
  static unsigned int *pool = nullptr;
  static int cursor = 0;
  static std::mutex mu;  // autograd's backward thread launches too
  std::lock_guard<std::mutex> lock(mu);
  if (!pool) {
    void *p = nullptr;
    if (hipGetSymbolAddress(&p, HIP_SYMBOL(g_handoff_pool)) != hipSuccess) return nullptr;
    pool = static_cast<unsigned int *>(p);
  }
  if (n <= 0 || n > HANDOFF_POOL) return nullptr;
  if (cursor + n > HANDOFF_POOL) cursor = 0;
  unsigned int *r = pool + cursor;
  cursor += (n + 63) & ~63;  // 256-B aligned ranges
  return r;
}

}  // namespace e2ep
