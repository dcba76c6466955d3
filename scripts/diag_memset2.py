"""hipMemsetAsync captured into a HIP graph (torch.cuda.graph) — replayed or not?"""
import ctypes

import torch

hip = ctypes.CDLL("libamdhip64.so")
hip.hipMemsetAsync.argtypes = [ctypes.c_void_p, ctypes.c_int, ctypes.c_size_t, ctypes.c_void_p]
hip.hipMemsetD32Async.argtypes = [ctypes.c_void_p, ctypes.c_int, ctypes.c_size_t, ctypes.c_void_p]
for nbytes in (4, 8, 12, 16, 64, 100, 256, 1024, 4096, 65536):
    buf = torch.full((nbytes,), 7, dtype=torch.uint8, device="cuda")
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        rc = hip.hipMemsetAsync(ctypes.c_void_p(buf.data_ptr()), 0, nbytes,
                                ctypes.c_void_p(torch.cuda.current_stream().cuda_stream))
        buf.add_(1)  # a kernel after the memset, like the reduction that uses it
    res = []
    for r in range(3):
        g.replay()
        torch.cuda.synchronize()
        res.append(int(buf.max()))
    print(nbytes, "rc", rc, "max after replays (want 1):", res, flush=True)
