"""Per-step random draws.

Every dropout on the path (attention probabilities, feed-forward ReLU, the LayerNorm residual
dropouts) draws its keep bits from a counter hash keyed by a device int32 seed
(csrc/dropout.h).  Instead of one torch.randint launch per dropout call (40 per train
step), `begin_step()` draws a pool of seeds at the start of a training forward and `seed()`
hands out views into it; the forward's other uniform draws (EfficientNet drop-connect, the
target-point noise) come from a float pool of the same launch (`uniform()`).  The launch is
e2ep_rng_draw: a splitmix64 hash of a per-device (seed, counter) state that the kernel itself
advances, so under HIP-graph capture every replay draws fresh values.  The state's seed comes
from torch's host generator when it is created (torch.manual_seed makes runs repeatable).
"""
import torch

from . import _lib

POOL = 64      # int32 dropout seeds per step
FPOOL = 2048   # uniform floats per step (drop-connect: blocks x images; noise: 2 x samples)
_pool = None
_next = 0
_fpool = None
_fnext = 0
_state = {}    # device -> int64 [seed, counter] device tensor


def _device_state(device):
    dev = torch.device(device)
    st = _state.get(dev)
    if st is None:
        if torch.cuda.is_current_stream_capturing():
            return None  # created on the first eager step; a capture-only process keeps torch's draws
        seed = int(torch.randint(0, 2 ** 62, (1,)).item())
        st = torch.tensor([seed, 0], dtype=torch.int64, device=dev)
        _state[dev] = st
    return st


def begin_step(device):
    """Draw this step's seed pool and uniform pool (one launch)."""
    global _pool, _next, _fpool, _fnext
    st = _device_state(device) if torch.device(device).type == "cuda" else None
    if st is None:
        _pool = torch.randint(0, 2 ** 31 - 1, (POOL,), dtype=torch.int32, device=device)
        _fpool = None
    else:
        _pool = torch.empty(POOL, dtype=torch.int32, device=device)
        _fpool = torch.empty(FPOOL, dtype=torch.float32, device=device)
        _lib.call("e2ep_rng_draw", _lib.ptr(st), FPOOL, _lib.ptr(_fpool), POOL, _lib.ptr(_pool),
                  _lib.stream())
    _next = 0
    _fnext = 0


def seed(device):
    """A (1,) int32 device seed for one dropout call: the next pool entry of this step, or a
    fresh draw when no pool is active (calls outside a training forward)."""
    global _next
    if _pool is None or _next >= POOL or _pool.device != torch.device(device):
        return torch.randint(0, 2 ** 31 - 1, (1,), dtype=torch.int32, device=device)
    s = _pool[_next:_next + 1]
    _next += 1
    return s


def uniform(shape, device, dtype=torch.float32):
    """torch.rand(shape) on the device: a view of this step's uniform pool when one is active
    and has room, else a torch draw."""
    global _fnext
    n = 1
    for d in shape:
        n *= int(d)
    if (_fpool is None or dtype != torch.float32 or _fnext + n > FPOOL
            or _fpool.device != torch.device(device)):
        return torch.rand(*shape, dtype=dtype, device=device)
    u = _fpool[_fnext:_fnext + n].view(*shape)
    _fnext += n
    return u


def end_step():
    """Retire the pools: later calls (outside a training forward) draw fresh values again, so
    a graph captured after this step does not bake in views of this step's pools."""
    global _pool, _next, _fpool, _fnext
    _pool = None
    _next = 0
    _fpool = None
    _fnext = 0
