"""Fused flat Adam (csrc/adam.hip) vs torch.optim.Adam (the reference's optimizer,
trainer/pl_trainer.py:116-121), fp32.  The update arithmetic is the same sequence of fp32
operations; contraction choices differ, so parameters agree to ~1e-7 relative."""
import pytest
import torch

from helpers import rel_l2

pytestmark = pytest.mark.gpu
DEV = "cuda"
SHAPES = [(5,), (64, 3, 3, 3), (4097,), (3, 7), (1, 10, 258), (20000,), (24,)]


def _params(seed):
    g = torch.Generator().manual_seed(seed)
    return [torch.randn(s, generator=g).to(DEV).requires_grad_() for s in SHAPES]


def _grads(step, skip=None):
    g = torch.Generator().manual_seed(100 + step)
    return [None if i == skip else torch.randn(s, generator=g).to(DEV) for i, s in enumerate(SHAPES)]


@pytest.mark.parametrize("wd", [0.0, 1e-4])
def test_flat_adam_matches_torch_adam(wd):
    from e2ep_amd.optim import FlatAdam
    ref, mine = _params(0), _params(0)
    topt = torch.optim.Adam(ref, lr=1e-3, weight_decay=wd, foreach=False)
    fopt = FlatAdam(mine, lr=1e-3, weight_decay=wd)
    for k in range(6):
        gs = _grads(k)
        for p, q, g in zip(ref, mine, gs):
            p.grad = g.clone()
            q.grad = g.clone()
        topt.step()
        fopt.prepare()
        fopt.step()
    for p, q in zip(ref, mine):
        assert rel_l2(q.detach(), p.detach()) < 1e-6
    # Adam-format state round trip
    sd = fopt.state_dict()
    tsd = topt.state_dict()
    for i in range(len(SHAPES)):
        assert float(sd["state"][i]["step"]) == float(tsd["state"][i]["step"])
        assert rel_l2(sd["state"][i]["exp_avg_sq"], tsd["state"][i]["exp_avg_sq"]) < 1e-6
    f2 = FlatAdam(_params(0), lr=1e-3, weight_decay=wd)
    f2.load_state_dict(tsd)
    assert rel_l2(f2.exp_avg, fopt.exp_avg) < 1e-6


def test_flat_adam_views_and_missing_grad():
    from e2ep_amd.optim import FlatAdam
    ps = _params(1)
    before = [p.detach().clone() for p in ps]
    opt = FlatAdam(ps, lr=1e-2)
    for p, b in zip(ps, before):  # parameters now live in the flat buffer, values unchanged
        assert torch.equal(p.detach(), b)
        assert p.data_ptr() % 16 == 0
    for p, g in zip(ps, _grads(0, skip=2)):
        p.grad = g
    opt.prepare()
    opt.step()
    assert torch.equal(ps[2].detach(), before[2])  # no gradient: not stepped (as torch)
    assert not torch.equal(ps[0].detach(), before[0])
    # torch.optim.Adam keeps no state for a tensor that was never stepped
    ref = _params(1)
    topt = torch.optim.Adam(ref, lr=1e-2)
    for p, g in zip(ref, _grads(0, skip=2)):
        p.grad = g
    topt.step()
    assert sorted(opt.state_dict()["state"]) == sorted(topt.state_dict()["state"]) == [
        i for i in range(len(SHAPES)) if i != 2]


def test_flat_adam_gathered_grads_equal_table_grads():
    """Data-parallel form: gather -> (all-reduce sum of 2 identical ranks) -> scale 1/2."""
    from e2ep_amd.optim import FlatAdam
    a, b = _params(2), _params(2)
    oa, ob = FlatAdam(a, lr=1e-3, weight_decay=1e-4), FlatAdam(b, lr=1e-3, weight_decay=1e-4)
    flat = torch.zeros(ob.numel, device=DEV)
    for k in range(3):
        gs = _grads(k)
        for p, q, g in zip(a, b, gs):
            p.grad, q.grad = g.clone(), g.clone()
        oa.prepare()
        oa.step()
        ob.prepare()
        ob.gather_grads(flat)
        flat.mul_(2.0)  # the all-reduce sum over two ranks with the same gradient
        ob.step(flat, 0.5)
    for p, q in zip(a, b):
        assert torch.equal(p.detach(), q.detach())
