"""Segmented backward (e2ep_amd.segments) on CPU tensors: cutting the forward and running the
backward in two stages gives every gradient bit for bit as one backward does, and the
gradient that crosses the cut keeps its layout (no re-layout copy; the BEV gradient crosses
it channels-last in the model)."""
import torch

from e2ep_amd import segments


class _ChannelsLastGrad(torch.autograd.Function):
    """Identity whose backward hands back a channels-last gradient (as the BEV stem does)."""

    @staticmethod
    def forward(ctx, x):
        return x.clone()

    @staticmethod
    def backward(ctx, g):
        return g.contiguous(memory_format=torch.channels_last)


def _net():
    torch.manual_seed(0)
    return (torch.nn.Conv2d(3, 8, 3, padding=1), torch.nn.Conv2d(8, 8, 3, padding=1),
            torch.nn.Linear(8 * 6 * 6, 5))


def _loss(mods, x, cut):
    c1, c2, lin = mods
    a = c1(x)                        # "camera encoder"
    side = a.mean(dim=(2, 3))        # a second output crossing the cut (pred_depth's role)
    a, side = cut(a), cut(side)
    b = _ChannelsLastGrad.apply(a)   # "BEV encoder" consuming the cut
    y = lin(torch.relu(c2(b)).flatten(1))
    return y.square().mean() + side.square().sum()


def _grads(mods):
    return [p.grad.clone() for m in mods for p in m.parameters()]


def test_two_stage_backward_equals_one_backward():
    x = torch.randn(2, 3, 6, 6)
    mods = _net()
    _loss(mods, x, lambda t: t).backward()
    want = _grads(mods)

    mods = _net()
    with segments.record() as rec:
        loss = _loss(mods, x, segments.cut)
    assert len(rec.pairs) == 2
    loss.backward()
    c1 = mods[0]
    assert c1.weight.grad is None  # stage 1 stops at the cut
    assert all(p.grad is not None for m in mods[1:] for p in m.parameters())
    (a, slot_a), (side, slot_s) = rec.pairs
    assert slot_a[0].is_contiguous(memory_format=torch.channels_last)  # layout kept
    assert not slot_a[0].is_contiguous()
    segments.backward_rest(rec.pairs)
    got = _grads(mods)
    assert all(torch.equal(g, w) for g, w in zip(got, want))


def test_cut_is_identity_outside_record():
    t = torch.randn(3, requires_grad=True)
    assert segments.cut(t) is t
    with segments.record() as rec:
        u = torch.randn(3)  # no gradient: not a cut point
        assert segments.cut(u) is u
    assert rec.pairs == []


def test_stage2_touching_a_stage1_gradient_is_detected():
    """The segmented graph step all-reduces stage-1 gradients before stage 2 runs; a parameter
    used on both sides of the cut (a shared weight) would be all-reduced before stage 2 adds
    its share.  segments.stage2_leaves_stage1 sees it (TrainStep then captures one backward)."""
    torch.manual_seed(0)
    lin_lo, lin_hi = torch.nn.Linear(4, 4), torch.nn.Linear(4, 1)
    shared = torch.nn.Parameter(torch.randn(4))
    x = torch.randn(3, 4)
    for share in (False, True):
        for p in (*lin_lo.parameters(), *lin_hi.parameters(), shared):
            p.grad = None
        with segments.record() as rec:
            a = lin_lo(x * shared) if share else lin_lo(x)   # below the cut
            a = segments.cut(a)
            loss = lin_hi(torch.tanh(a) * shared).sum()       # above the cut (stage 1)
        loss.backward()
        stage1 = [shared, *lin_hi.parameters()]
        marks = segments.grad_marks(stage1)
        segments.backward_rest(rec.pairs)
        assert segments.stage2_leaves_stage1(stage1, marks) == (not share)


def test_train_step_rig_key_compares_rig_values():
    """TrainStep's captured-rig check (e2ep_amd.train._rig_key): a rig is identified by its
    shapes and fp32 bytes, whatever its device or dtype, so a graph-mode step refuses a batch
    whose rig differs from the captured one and accepts an equal one (reference rig handling:
    model/bev_model.py:45-57; the captured plan is the rig's)."""
    from e2ep_amd.train import _rig_key
    K = torch.eye(3).repeat(2, 4, 1, 1)
    E = torch.eye(4).repeat(2, 4, 1, 1)
    k0 = _rig_key({"intrinsics": K, "extrinsics": E})
    assert k0 == _rig_key({"intrinsics": K.clone().double(), "extrinsics": E.clone()})
    E2 = E.clone()
    E2[0, 0, 0, 3] += 0.25
    assert k0 != _rig_key({"intrinsics": K, "extrinsics": E2})
    assert k0 != _rig_key({"intrinsics": K[:1], "extrinsics": E[:1]})
    assert _rig_key({"image": torch.zeros(1)}) is None
