"""Per-step dropout seeds.

Every dropout on the path (attention probabilities, feed-forward ReLU, the LayerNorm residual
dropouts) draws its keep bits from a counter hash keyed by a device int32 seed
(csrc/dropout.h).  Instead of one torch.randint launch per dropout call (40 per train
step), `begin_step()` draws a pool of seeds with ONE launch at the start of a training
forward and `seed()` hands out views into it.  Under HIP-graph capture the pool draw is
captured with the step, so every replay gets fresh seeds for every call site.
"""
import torch

POOL = 64
_pool = None
_next = 0


def begin_step(device):
    """Draw this step's seed pool (one launch)."""
    global _pool, _next
    _pool = torch.randint(0, 2 ** 31 - 1, (POOL,), dtype=torch.int32, device=device)
    _next = 0


def seed(device):
    """A (1,) int32 device seed for one dropout call: the next pool entry of this step, or a
    fresh draw when no pool is active (calls outside a training forward)."""
    global _next
    if _pool is None or _next >= POOL or _pool.device != torch.device(device):
        return torch.randint(0, 2 ** 31 - 1, (1,), dtype=torch.int32, device=device)
    s = _pool[_next:_next + 1]
    _next += 1
    return s


def end_step():
    """Retire the pool: later calls (outside a training forward) draw fresh seeds again, so a
    graph captured after this step does not bake in a view of this step's pool."""
    global _pool, _next
    _pool = None
    _next = 0
