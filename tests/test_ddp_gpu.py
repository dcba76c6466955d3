"""Data-parallel and LR-schedule paths of TrainStep on one MI355X.

* The LR a captured step uses is a device scalar (FlatAdam.lr_dev): CosineAnnealingLR
  (reference trainer/pl_trainer.py:120) changes it between replays exactly as it changes an
  eager step.
* RCCL at world 1 (the exchange is an identity): the graph-mode step (backward in two
  captured segments, the stage-1 buckets' all-reduces issued between the segment replays so
  they overlap the stage-2 backward, captured Adam) and the eager step with the bucketed,
  hook-driven all-reduce overlapping backward both give the same parameters as the step
  without an exchange, bit for bit.
* gloo at world 2, both ranks on cuda:0 (the one-GPU rehearsal of the N>1 path): the default
  graph-mode exchange — the segmented backward with the stage-1 buckets exchanged while stage 2
  runs, each bucket staged through pinned host memory — of the real ParkingModel TrainStep,
  rank r training on its OWN batch (synthetic seed 7 + r, target noise 7 + r), equals the
  data-parallel step computed in one process (each rank's batch through the same weights, BN
  batch statistics per rank as DDP without SyncBN, the two flat gradients summed and one
  FlatAdam.step(sum, 1/2)) and the single-graph exchange (segment=False), bit for bit; and the
  check can fail: skipping the all-reduce of one stage-1 bucket (a test-only switch) breaks it.
  Reference: pl_train.py:42-47 (DDP when num_gpus > 1).
"""
import os
import socket

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from helpers import rel_l2

pytestmark = pytest.mark.gpu
DEV = "cuda"


class _Small(torch.nn.Module):
    def __init__(self):
        super().__init__()
        torch.manual_seed(3)
        self.a = torch.nn.Linear(16, 32)
        self.b = torch.nn.Linear(32, 4)

    def training_step(self, batch, idx=0):
        return (self.b(self.a(batch["x"]).relu()) - batch["y"]).pow(2).mean()


def _small_batch():
    g = torch.Generator().manual_seed(1)
    return {"x": torch.randn(8, 16, generator=g).to(DEV), "y": torch.randn(8, 4, generator=g).to(DEV)}


def test_lr_schedule_follows_under_graph_replay():
    from e2ep_amd.optim import FlatAdam
    from e2ep_amd.train import TrainStep
    runs = {}
    for graph in (False, True):
        m = _Small().to(DEV)
        opt = FlatAdam([p for p in m.parameters()], lr=1e-2, weight_decay=1e-4)
        sched = torch.optim.lr_scheduler.CosineAnnealingLR(opt, T_max=4)
        step = TrainStep(m, _small_batch(), graph=graph, warmup=1, optimizer=opt)
        if not graph:
            step()  # the graph run's one warm-up step (initial LR)
        lrs = []
        for _ in range(4):
            step()
            lrs.append(opt.param_groups[0]["lr"])
            sched.step()
        runs[graph] = (torch.cat([p.detach().reshape(-1) for p in m.parameters()]), lrs,
                       float(opt.lr_dev))
    (pe, lre, _), (pg, lrg, dev_lr) = runs[False], runs[True]
    assert lre == lrg and lre[0] != lre[2]
    assert dev_lr == lrg[-1]  # the device scalar the last replay read
    assert rel_l2(pg, pe) < 1e-6
    # LR 0 under replay: the captured Adam launch must not move the weights
    m = _Small().to(DEV)
    opt = FlatAdam(list(m.parameters()), lr=1e-2)
    step = TrainStep(m, _small_batch(), graph=True, warmup=1, optimizer=opt)
    step()
    opt.param_groups[0]["lr"] = 0.0
    before = torch.cat([p.detach().reshape(-1) for p in m.parameters()]).clone()
    step()
    after = torch.cat([p.detach().reshape(-1) for p in m.parameters()])
    assert torch.equal(before, after)
    opt.param_groups[0]["lr"] = 1e-2
    step()
    assert not torch.equal(after, torch.cat([p.detach().reshape(-1) for p in m.parameters()]))


def _port():
    with socket.socket() as so:
        so.bind(("127.0.0.1", 0))
        return so.getsockname()[1]


def _parking_module(seed_noise=7):
    from e2ep_amd import synthetic
    from trainer.pl_trainer import ParkingTrainingModule
    from tool.config import default_cfg
    from weights import make_state
    mod = ParkingTrainingModule(default_cfg(deterministic=True))
    mod.parking_model.load_state_dict(make_state(mod.parking_model.state_dict(), 1234))
    mod = mod.to(DEV).train()
    for p in mod.parking_model.bev_encoder.layer4.parameters():
        p.requires_grad_(False)
    noise = synthetic.target_noise(1, seed=seed_noise).to(DEV)
    mod.parking_model._noise = lambda b, device, n: noise
    return mod


def _parking_batch():
    from e2ep_amd import synthetic
    d = synthetic.synthetic_batch(1, seed=7)
    return {k: (v if k in ("intrinsics", "extrinsics") else v.to(DEV)) for k, v in d.items()}


def _flat_params(mod):
    return torch.cat([p.detach().reshape(-1) for p in mod.parameters()]).cpu()


@pytest.mark.parametrize("graph", [True, False])
def test_rccl_world1_exchange_is_exact(graph):
    from e2ep_amd.train import TrainStep
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(_port()))
    dist.init_process_group("nccl", rank=0, world_size=1, device_id=torch.device(DEV, 0))
    try:
        m_ref, m_ddp = _parking_module(), _parking_module()
        s_ref = TrainStep(m_ref, _parking_batch(), graph=graph, warmup=1)
        s_ddp = TrainStep(m_ddp, _parking_batch(), graph=graph, warmup=1, ddp=True, bucket_mb=4.0)
        if graph:
            # segmented backward: >= 4 buckets, most of them issued before stage 2 runs
            assert s_ddp.buckets is None and s_ddp.segmented and s_ddp.g_bwd is None
            b1, b2 = s_ddp.seg_buckets
            assert len(b1) + len(b2) >= 4 and len(b1) >= 3 and len(b2) >= 1
            spans = sorted(b1 + b2)
            assert spans[0][0] == 0 and spans[-1][1] == s_ddp.flat_grad.numel()
            assert all(a[1] == b[0] for a, b in zip(spans, spans[1:]))  # a partition
        else:
            assert s_ddp.buckets is not None and len(s_ddp.buckets.buckets) >= 10
        for _ in range(3):
            l_ref, l_ddp = float(s_ref()), float(s_ddp())
            assert l_ref == l_ddp
        assert torch.equal(_flat_params(m_ref), _flat_params(m_ddp))
    finally:
        torch.cuda.synchronize()  # no queued work on any stream when the communicator goes
        dist.destroy_process_group()


def _rank_batch(rank):
    from e2ep_amd import synthetic
    d = synthetic.synthetic_batch(1, seed=7 + rank)
    return {k: (v if k in ("intrinsics", "extrinsics") else v.to(DEV)) for k, v in d.items()}


_STEPS = 2  # replays after the one eager warm-up step


def _gloo_worker(rank, world, port, out):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    torch.cuda.set_device(0)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from e2ep_amd.train import TrainStep
    for case in ("segmented", "single", "skip"):
        segment = case != "single"
        m = _parking_module(seed_noise=7 + rank)
        s = TrainStep(m, _rank_batch(rank), world=world, graph=True, warmup=1, bucket_mb=4.0,
                      segment=segment)
        assert s.buckets is None and s._host is not None
        if segment:  # the default graph-mode exchange: stage buckets between segment replays
            assert s.segmented and s.g_bwd is None and s.g_s2 is not None
            b1, b2 = s.seg_buckets
            assert len(b1) >= 3 and len(b2) >= 1
            spans = sorted(b1 + b2)
            assert spans[0][0] == 0 and spans[-1][1] == s.flat_grad.numel()
            assert all(a[1] == b[0] for a, b in zip(spans, spans[1:]))  # a partition
        else:
            assert not s.segmented and s.g_bwd is not None and s.g_gather is not None
        if case == "skip":
            s._test_skip = (0, 0)  # the first stage-1 bucket is never exchanged
        losses = [float(s()) for _ in range(_STEPS)]
        out[(rank, case)] = (losses, _flat_params(m))
        del s, m
    dist.destroy_process_group()


def _one_process_data_parallel(steps):
    """The world-2 step in one process: both ranks' batches through the same weights (one
    module; BN normalises each forward with its own batch statistics, as per-rank BN under
    DDP does), each rank's gradients gathered into a flat buffer, the all-reduce's sum
    formed, and one FlatAdam.step(sum, 1/world) — steps times, the first one eager like
    TrainStep's warm-up.  Returns (losses per rank, flat parameters)."""
    from e2ep_amd import synthetic
    from e2ep_amd.optim import FlatAdam
    m = _parking_module()
    params = [p for p in m.parameters() if p.requires_grad]
    opt = FlatAdam(params, lr=1e-4, weight_decay=1e-4)  # TrainStep's defaults
    batches = [_rank_batch(r) for r in range(2)]
    noises = [synthetic.target_noise(1, seed=7 + r).to(DEV) for r in range(2)]
    flats = [torch.zeros(opt.numel, device=DEV) for _ in range(2)]
    has = [torch.zeros(len(params), dtype=torch.int64, device=DEV) for _ in range(2)]
    one = torch.ones((), device=DEV)
    losses = {0: [], 1: []}
    for _ in range(steps):
        for r in range(2):
            m.parking_model._noise = lambda b, device, n, z=noises[r]: z
            opt.zero_grad(set_to_none=True)
            loss = m.training_step(batches[r], 0)
            loss.backward(one)
            opt.prepare()
            opt.gather_grads(flats[r])
            opt.has_grad(has[r])
            losses[r].append(float(loss))
        opt.step(flats[0] + flats[1], 0.5, has_grad=torch.maximum(has[0], has[1]))
    torch.cuda.synchronize()
    return losses, _flat_params(m)


def test_gloo_two_rank_rehearsal_equals_one_process():
    want_losses, want = _one_process_data_parallel(1 + _STEPS)
    with mp.Manager() as man:
        out = man.dict()
        mp.spawn(_gloo_worker, args=(2, _port(), out), nprocs=2, join=True)
        res = dict(out)
    (l0, p0), (l1, p1) = res[(0, "segmented")], res[(1, "segmented")]
    (l0s, p0s), (l1s, p1s) = res[(0, "single")], res[(1, "single")]
    # each rank saw its own batch: different losses, identical replicas afterwards
    assert l0 != l1 and l0[0] != l1[0]
    assert l0 == want_losses[0][1:] and l1 == want_losses[1][1:]
    assert l0s == l0 and l1s == l1
    assert torch.equal(p0, p1) and torch.equal(p0s, p1s)
    # the mean of two DIFFERENT gradients, through the segmented and the single-graph
    # exchange, equals the one-process data-parallel step (the bound asked for is 1e-6
    # relative; the sum of two fp32 values is order-free, so it holds bit for bit)
    assert rel_l2(p0, want) <= 1e-6 and torch.equal(p0, want)
    assert torch.equal(p0, p0s)
    # the check can fail: one stage-1 bucket not exchanged -> replicas drift apart and away
    # from the data-parallel step
    (_, pk0), (_, pk1) = res[(0, "skip")], res[(1, "skip")]
    assert not torch.equal(pk0, pk1)
    assert rel_l2(pk0, want) > 1e-6 and rel_l2(pk1, want) > 1e-6
