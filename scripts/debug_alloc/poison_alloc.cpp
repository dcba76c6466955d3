// Debug allocator for torch.cuda.memory.CUDAPluggableAllocator: every allocation is fresh
// memory filled with 0xFF (NaN as fp32) and every free poisons the block in stream order
// and never hands it out again, so a kernel that reads or writes a tensor after its
// release sees NaN instead of a recycled block.  Leaks by design (debug runs only).
#include <hip/hip_runtime.h>
#include <sys/types.h>

extern "C" {

void *e2ep_dbg_malloc(ssize_t size, int device, hipStream_t stream) {
  void *p = nullptr;
  hipSetDevice(device);
  if (hipMalloc(&p, size > 0 ? size : 1) != hipSuccess) return nullptr;
  if (size > 0) hipMemsetAsync(p, 0xFF, size, stream);
  return p;
}

void e2ep_dbg_free(void *ptr, ssize_t size, int device, hipStream_t stream) {
  hipSetDevice(device);
  if (size > 0) hipMemsetAsync(ptr, 0xFF, size, stream);
}

}  // extern "C"
