"""HIP-graph capture with the memset-node repair (csrc/graph.hip).

Memset nodes captured into a HIP graph replay correctly only on the first launch on this
ROCm stack, and PyTorch's reductions capture them (cross-block semaphores), so every graph
the train step captures is kept un-instantiated, its memset nodes are rewritten into
kernel nodes by e2ep_graph_replace_memsets, and only then instantiated."""
import ctypes

import torch

from . import _lib


def capture(fn, pool=None):
    """Capture fn() into a repaired, instantiated graph.  Returns (graph, fn's result,
    number of memset nodes rewritten)."""
    g = torch.cuda.CUDAGraph(keep_graph=True)
    # thread-local capture: other threads' HIP calls during the capture (the c10d watchdog
    # polling its RCCL work events when a process group exists) must neither invalidate the
    # capture nor be refused by it
    with torch.cuda.graph(g, pool=pool, capture_error_mode="thread_local"):
        out = fn()
    n = ctypes.c_int(0)
    _lib.call("e2ep_graph_replace_memsets", ctypes.c_void_p(g.raw_cuda_graph()), ctypes.byref(n))
    g.instantiate()
    return g, out, n.value
