"""N>1 data-parallel path of TrainStep on CPU: world_size 2 over gloo (127.0.0.1).

Each rank steps its own half of the batch; the bucketed, hook-driven all-reduce of the flat
gradient buffer (several buckets, issued during backward in the same order on every rank)
and the non-overlapped single all-reduce must both reproduce one step over the whole batch on
one process (DistributedDataParallel semantics, reference pl_train.py:47 strategy 'ddp').
A parameter that gets no gradient is not stepped on any rank (as torch.optim.Adam)."""
import os
import socket

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp


class _HostSGD:
    """Host stand-in for FlatAdam's interface (prepare / gather_grads / step with a flat,
    scaled gradient), so TrainStep's data-parallel orchestration runs on CPU ranks.  The
    HIP optimizer itself is covered by tests/test_optim_gpu.py."""

    def __init__(self, params, lr):
        self.params, self.lr = list(params), lr
        self.spans, off = [], 0
        for p in self.params:
            self.spans.append((off, p.numel()))
            off += (p.numel() + 3) // 4 * 4  # FlatAdam's 16-byte alignment pads
        self.numel = off
        self.had_grad = [False] * len(self.params)

    def zero_grad(self, set_to_none=True):
        for p in self.params:
            p.grad = None

    def prepare(self, params=None):
        i0, i1 = params if params is not None else (0, len(self.params))
        for i in range(i0, i1):
            self.had_grad[i] = self.params[i].grad is not None

    def has_grad(self, out):
        out.copy_(torch.tensor([p.grad is not None for p in self.params], dtype=out.dtype))
        return out

    def gather_grads(self, out, params=None):
        i0, i1 = params if params is not None else (0, len(self.params))
        for i in range(i0, i1):
            o, n = self.spans[i]
            g = self.params[i].grad
            out[o:o + n] = 0.0 if g is None else g.reshape(-1)

    @torch.no_grad()
    def step(self, grad_flat=None, grad_scale=1.0, has_grad=None):
        self.prepare()
        for i, p in enumerate(self.params):
            stepped = self.had_grad[i] if has_grad is None or grad_flat is None else bool(has_grad[i])
            if not stepped:
                continue  # no gradient: not stepped (FlatAdam's null table entry)
            o, n = self.spans[i]
            g = p.grad if grad_flat is None else grad_flat[o:o + n].view_as(p)
            p.sub_(self.lr * grad_scale * g)


class _Tiny(torch.nn.Module):
    def __init__(self):
        super().__init__()
        torch.manual_seed(0)
        self.conv = torch.nn.Conv2d(3, 4, 3, padding=1)
        self.head = torch.nn.Linear(4, 2)
        self.mid = torch.nn.Linear(4, 4)
        self.frozen = torch.nn.Linear(2, 2)  # no grad, like bev_encoder.layer4
        for p in self.frozen.parameters():
            p.requires_grad_(False)
        self.branch = torch.nn.Linear(4, 1)  # used only where self.use_branch (rank-dependent)
        self.unused = torch.nn.Linear(3, 3)  # trainable but never run: no gradient
        self.use_branch = False

    def training_step(self, batch, idx=0):
        h = self.conv(batch["x"]).relu().mean((2, 3))
        loss = torch.nn.functional.mse_loss(self.head(self.mid(h).relu() + h), batch["y"])
        if self.use_branch:
            loss = loss + 0.1 * self.branch(h).square().mean()
        return loss


def _data():
    g = torch.Generator().manual_seed(5)
    return {"x": torch.randn(4, 3, 8, 8, generator=g), "y": torch.randn(4, 2, generator=g)}


def _worker(rank, world, port, out, overlap, branch_rank=None):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from e2ep_amd.train import TrainStep
    d = _data()
    half = {k: v[rank * 2:(rank + 1) * 2] for k, v in d.items()}
    m = _Tiny()
    m.use_branch = rank == branch_rank
    params = [p for p in m.parameters() if p.requires_grad]
    # 64-byte buckets: one bucket per tensor or two, so several all-reduces run per step
    s = TrainStep(m, half, world=world, graph=False, optimizer=_HostSGD(params, 1e-2),
                  bucket_mb=64 / 2 ** 20, overlap=overlap)
    assert (s.buckets is not None) == overlap
    if overlap:
        assert len(s.buckets.buckets) >= 4
    for _ in range(3):
        s()
    out[rank] = torch.cat([p.detach().reshape(-1) for p in m.parameters()])
    dist.destroy_process_group()


def _port():
    with socket.socket() as so:
        so.bind(("127.0.0.1", 0))
        return so.getsockname()[1]


@pytest.mark.parametrize("overlap", [True, False])
def test_two_rank_step_equals_full_batch_step(overlap):
    from e2ep_amd.train import TrainStep
    ref = _Tiny()
    params = [p for p in ref.parameters() if p.requires_grad]
    s = TrainStep(ref, _data(), world=1, graph=False, optimizer=_HostSGD(params, 1e-2))
    for _ in range(3):
        s()
    want = torch.cat([p.detach().reshape(-1) for p in ref.parameters()])
    with mp.Manager() as man:
        out = man.dict()
        mp.spawn(_worker, args=(2, _port(), out, overlap), nprocs=2, join=True)
        got0, got1 = out[0], out[1]
    assert torch.equal(got0, got1)  # ranks stay in lock-step
    assert torch.allclose(got0, want, rtol=1e-5, atol=1e-6)
    assert torch.equal(ref.frozen.weight, _Tiny().frozen.weight)  # untouched
    n_unused = sum(p.numel() for p in ref.unused.parameters())
    assert torch.equal(got0[-n_unused:], torch.cat([p.detach().reshape(-1)
                                                    for p in _Tiny().unused.parameters()]))


@pytest.mark.parametrize("overlap", [True, False])
def test_rank_dependent_branch_steps_every_replica(overlap):
    """A parameter that gets a gradient on one rank only (a rank-dependent branch) is stepped
    on every rank with the averaged gradient, as under DDP: the replicas stay identical
    (the gradient-presence mask is all-reduced with the gradients)."""
    with mp.Manager() as man:
        out = man.dict()
        mp.spawn(_worker, args=(2, _port(), out, overlap, 1), nprocs=2, join=True)
        got0, got1 = out[0], out[1]
    assert torch.equal(got0, got1)
    init = _Tiny()
    nb = sum(p.numel() for p in init.branch.parameters())
    nu = sum(p.numel() for p in init.unused.parameters())
    start = torch.cat([p.detach().reshape(-1) for p in init.branch.parameters()])
    assert not torch.equal(got0[-(nu + nb):-nu], start)  # moved on rank 0 too
