"""Backward in segments: cut points in the forward, so a graph-captured data-parallel step can
all-reduce the gradients of the upper layers while the lower layers' backward still runs.

The reference's DDP overlaps bucketed gradient all-reduces with the backward
(pl_train.py:47, DistributedDataParallel's autograd hooks).  A captured collective is not an
option on this stack, and a single captured backward gives the host no point
at which to issue one.  Instead the forward is cut: at a cut point the activation `a` is
replaced downstream by a stand-in that does not lead back to `a`, so `loss.backward()` stops
there (stage 1: losses, heads, transformer, BEV encoder) and leaves d loss / d a in the cut's
slot; `torch.autograd.backward(a, d loss / d a)` then runs the rest (stage 2: lift-splat and
the camera encoder).  Every gradient is the same tensor, computed by the same kernels in the same
order, as one backward would give (tests/test_ddp_gpu.py checks this bit for bit).  Each stage
is its own HIP graph; between the replays the host issues the stage-1 buckets' RCCL
all-reduces on a communication stream, which then run concurrently with stage 2.

Cut points are declared in the model (`cut(t)`); outside `record()` they are the identity.
The stand-in is not a plain `detach().requires_grad_()` leaf: a leaf's AccumulateGrad would
re-lay-out a gradient whose strides differ from the leaf's (the BEV gradient arrives pillar-
major, channels-last, for the lift-splat backward) with an extra copy; the stand-in's
backward keeps the incoming gradient tensor as it is."""
import torch

_active = None
_anchor = {}


class record:
    """Collect the cut points of the forward run inside the block: `pairs` = [(a, slot)];
    after stage 1 `slot` holds d loss / d a (empty when nothing downstream used it)."""

    def __enter__(self):
        global _active
        _active = []
        self.pairs = _active
        return self

    def __exit__(self, *exc):
        global _active
        _active = None
        return False


class _Cut(torch.autograd.Function):
    @staticmethod
    def forward(ctx, anchor, x, slot):
        ctx.slot = slot
        return x.view_as(x)

    @staticmethod
    def backward(ctx, g):
        ctx.slot.append(g)
        return None, None, None


def ensure_anchor(device):
    """Create the device's anchor leaf now (call outside graph capture)."""
    if device not in _anchor:
        _anchor[device] = torch.zeros(0, device=device, requires_grad=True)


def cut(t):
    """Identity outside record(); inside, a stand-in for `t` whose gradient stops here."""
    if _active is None or not getattr(t, "requires_grad", False):
        return t
    anchor = _anchor.get(t.device)
    if anchor is None:  # a zero-element leaf that makes the stand-in require a gradient
        anchor = _anchor[t.device] = torch.zeros(0, device=t.device, requires_grad=True)
    slot = []
    _active.append((t, slot))
    return _Cut.apply(anchor, t.detach(), slot)


def backward_rest(pairs):
    """Stage 2: propagate the gradient each stand-in received into the segment above it."""
    outs = [a for a, slot in pairs if slot]
    if outs:
        torch.autograd.backward(outs, [slot[0] for a, slot in pairs if slot])


def grad_marks(params):
    """(gradient tensor id, storage address, version counter) of each parameter's .grad (None
    when it has none): what a later backward changes when it accumulates into a gradient — in
    place (version), or by handing autograd's result over (a new tensor)."""
    return [None if p.grad is None else (id(p.grad), p.grad.data_ptr(), p.grad._version)
            for p in params]


def stage2_leaves_stage1(params, marks):
    """True when the stage-2 backward left the stage-1 gradients (`params`, their marks taken
    after stage 1) untouched.  A parameter used on both sides of a cut (shared weights) would
    have its stage-1 gradient gathered and all-reduced before stage 2 adds its share, and the
    step would train on wrong gradients — the segmented capture falls back to one backward
    graph instead."""
    return grad_marks(params) == marks
