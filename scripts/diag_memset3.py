"""Which HIP memory nodes replay correctly from a captured graph?"""
import ctypes

import torch

hip = ctypes.CDLL("libamdhip64.so")
vp, sz, i = ctypes.c_void_p, ctypes.c_size_t, ctypes.c_int
hip.hipMemsetAsync.argtypes = [vp, i, sz, vp]
hip.hipMemsetD32Async.argtypes = [vp, i, sz, vp]
hip.hipMemsetD8Async.argtypes = [vp, ctypes.c_ubyte, sz, vp]
hip.hipMemcpyAsync.argtypes = [vp, vp, sz, i, vp]
HIP_D2D = 3


def stream():
    return vp(torch.cuda.current_stream().cuda_stream)


def case(name, op, n=4096):
    buf = torch.full((n,), 7, dtype=torch.int32, device="cuda")
    src = torch.zeros(n, dtype=torch.int32, device="cuda")
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        op(buf, src)
        buf.add_(1)
    res = []
    for _ in range(3):
        g.replay()
        torch.cuda.synchronize()
        res.append((int(buf.min()), int(buf.max())))
    print(f"{name:24s} (min,max) per replay, want (1,1):", res, flush=True)


case("hipMemsetAsync", lambda b, s: hip.hipMemsetAsync(vp(b.data_ptr()), 0, b.numel() * 4, stream()))
case("hipMemsetD32Async", lambda b, s: hip.hipMemsetD32Async(vp(b.data_ptr()), 0, b.numel(), stream()))
case("hipMemsetD8Async", lambda b, s: hip.hipMemsetD8Async(vp(b.data_ptr()), 0, b.numel() * 4, stream()))
case("hipMemcpyAsync D2D", lambda b, s: hip.hipMemcpyAsync(vp(b.data_ptr()), vp(s.data_ptr()), b.numel() * 4, HIP_D2D, stream()))
case("torch copy_", lambda b, s: b.copy_(s))
case("torch zero_", lambda b, s: b.zero_())
case("torch clone->copy", lambda b, s: b.copy_(s.clone()))
