"""HIP-graph capture with the memset-node repair (csrc/graph.hip).

Memset nodes captured into a HIP graph replay correctly only on the first launch on this
ROCm stack, and PyTorch's reductions capture them (cross-block semaphores), so every graph
the train step captures is kept un-instantiated, its memset nodes are rewritten into
kernel nodes by e2ep_graph_replace_memsets, and only then instantiated."""
import ctypes
import os
import sys

import torch
import torch.distributed as dist
from torch.utils._python_dispatch import TorchDispatchMode

from . import _lib

_DEBUG = os.environ.get("E2EP_CAPTURE_DEBUG", "0") == "1"  # per-stream join-check report on stderr


def capture_mode():
    """'thread_local' while a process group exists, else 'global'.

    With a process group the c10d watchdog thread polls its RCCL work events during a
    capture; under the global mode those calls race with (and invalidate) the capture — in
    round 2 an abort inside destroy_process_group after the world-1 RCCL test.
    Without one, the global mode is kept: it makes any unsafe HIP call from another thread
    (autograd's device thread runs the captured backward) fail the capture loudly instead of
    being captured or skipped silently."""
    return "thread_local" if dist.is_available() and dist.is_initialized() else "global"


class _SeededOps(TorchDispatchMode):
    """Records the aten ops tagged nondeterministic_seeded (torch.rand, dropout, bernoulli_,
    ...) that run while a graph is captured: they draw from torch's generators, whose state a
    captured graph reads from the per-replay prologue of torch.cuda.CUDAGraph.replay()."""

    def __init__(self):
        super().__init__()
        self.seen = []

    def __torch_dispatch__(self, func, types, args=(), kwargs=None):
        if torch.Tag.nondeterministic_seeded in func.tags:
            self.seen.append(str(func))
        return func(*args, **(kwargs or {}))


class Graph:
    """A captured, repaired graph with its own executable (e2ep_graph_exec_*): replay()
    launches it on the current stream without torch.cuda.CUDAGraph.replay()'s prologue, which
    refreshes torch's generator states with int64 fill kernels before every launch (the step
    draws its random numbers from e2ep_rng_draw, not from torch's generators).  The torch
    graph object stays alive: it owns the graph and its memory pool.

    A capture that drew from torch's generators (`torch_rng`: e.g. a user module's nn.Dropout,
    or rng.py's torch fallbacks when no step pool is active) replays through torch's own
    replay instead, whose prologue advances the generator offsets, so those draws differ from
    replay to replay as they would eagerly."""

    def __init__(self, g, torch_rng=()):
        self.g = g
        self.torch_rng = tuple(torch_rng)
        self._exec = None
        if self.torch_rng:
            g.instantiate()  # torch's executable of the repaired graph
            return
        ex = ctypes.c_void_p()
        _lib.call("e2ep_graph_exec_create", ctypes.c_void_p(g.raw_cuda_graph()), ctypes.byref(ex))
        self._exec = ex

    def replay(self):
        if self._exec is None:
            self.g.replay()
            return
        _lib.call("e2ep_graph_exec_launch", self._exec, _lib.stream())

    def pool(self):
        return self.g.pool()

    def __del__(self):
        try:
            if self._exec:
                _lib.call("e2ep_graph_exec_destroy", self._exec)
        except Exception:  # noqa: BLE001 - interpreter shutdown
            pass


def _side_streams():
    """(name, stream) of every side stream the product forks inside a capture: the model
    branches (streams.py) and the weight-gradient forks (conv._Fork)."""
    from . import conv, streams
    out = [("branch '%s' (device %d)" % (k[1], k[0]), st) for k, st in streams._STREAMS.items()]
    out += [("weight-gradient side stream of stream 0x%x (device %d)" % (k[1], k[0]), st)
            for k, st in conv._SIDE.items()]
    return out


def _join_check():
    """Inside a capture, after the captured work: every side stream that took part in the
    capture must have rejoined the origin stream (its last work an ancestor of the origin's
    frontier).  An unjoined one is joined here, so the capture can still end cleanly, and
    named in the E2EPError the caller raises (a nested fork once made hipStreamEndCapture
    segfault instead: streams.py)."""
    origin = torch.cuda.current_stream()
    bad = []
    for name, st in _side_streams():
        if st.device != origin.device or st == origin:
            continue
        u = ctypes.c_int(0)
        _lib.call("e2ep_capture_unjoined", ctypes.c_void_p(origin.cuda_stream),
                  ctypes.c_void_p(st.cuda_stream), ctypes.byref(u))
        if _DEBUG:
            print(f"graphs.capture join check: {name}: {'UNJOINED' if u.value else 'joined / not in the capture'}",
                  file=sys.stderr, flush=True)
        if u.value:
            origin.wait_stream(st)
            bad.append(name)
    return bad


def capture(fn, pool=None):
    """Capture fn() into a repaired graph with its own executable (torch's, when fn drew from
    torch's generators: Graph).  Returns (Graph, fn's result, number of memset nodes
    rewritten).  Raises E2EPError when fn left a forked side stream unjoined."""
    g = torch.cuda.CUDAGraph(keep_graph=True)
    seeded = _SeededOps()
    with torch.cuda.graph(g, pool=pool, capture_error_mode=capture_mode()):
        with seeded:
            out = fn()
        unjoined = _join_check()
    if unjoined:
        raise _lib.E2EPError("graphs.capture: side stream(s) forked inside the capture never "
                             "rejoined the capturing stream: " + "; ".join(unjoined))
    n = ctypes.c_int(0)
    _lib.call("e2ep_graph_replace_memsets", ctypes.c_void_p(g.raw_cuda_graph()), ctypes.byref(n))
    return Graph(g, seeded.seen), out, n.value
