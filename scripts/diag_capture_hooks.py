"""Diagnostic (verdict r2, weak #7): the round-2 data-parallel graph design ran the bucket
gathers + all-reduces from post-accumulate-grad hooks on a side stream INSIDE the captured
backward, and replayed wrong camera-encoder gradients (profiles/r02/ddp_diag/diag_ddp2.log:
386 of 530 tensors wrong with the collective stubbed out, so not RCCL).  This re-runs that
configuration (TrainStep(overlap="captured"), all_reduce stubbed) under today's capture mode
and varies one factor at a time:
  A  as round 2: the gathers' device gradient table still holds the LAST EAGER WARM-UP
     step's gradient addresses (round 2 re-pointed it only after the step; those tensors were
     freed by zero_grad(set_to_none) at the start of the captured step, and the capture's own
     gradients live elsewhere in the graph pool); conv weight gradients forked (conv._Fork)
  B  as A with the conv weight-gradient fork off
  C  as A, but the table re-pointed at the captured gradients after capture, before replay
     (what TrainStep does for its non-hook gather graph)
Each prints how many parameter gradients differ from a plain captured step (no hooks)."""
import os
import socket
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "e2e-parking-carla_amd"), ROOT, os.path.join(ROOT, "tests")]
import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402


def port():
    with socket.socket() as so:
        so.bind(("127.0.0.1", 0))
        return so.getsockname()[1]


os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port()))
dist.init_process_group("nccl", rank=0, world_size=1, device_id=torch.device("cuda", 0))

from test_ddp_gpu import _parking_batch, _parking_module  # noqa: E402
import e2ep_amd.train as T  # noqa: E402
from e2ep_amd import conv  # noqa: E402
from e2ep_amd.train import TrainStep  # noqa: E402


class _Done:
    def wait(self):
        pass


real_ar = dist.all_reduce
real_finish = T.GradBuckets.finish
real_capture = T.graphs.capture


def finish_round2(self):
    """GradBuckets.finish without its final table update while capturing (as in round 2)."""
    while self.next < len(self.buckets):
        self._launch(self.next)
        self.next += 1
    for w in self.works:
        w.wait()
    self.main.wait_stream(self.comm)
    if not self.capturing:
        self.opt.prepare()


def run(tag, wgrad_fork, reprepare, hooks=True):
    from e2ep_amd.optim import FlatAdam
    conv._OVERLAP[0] = wgrad_fork
    T.GradBuckets.finish = finish_round2
    dist.all_reduce = lambda t, async_op=False, **k: _Done()
    saved = {}
    try:
        m_ref, m_ddp = _parking_module(), _parking_module()
        s_ref = TrainStep(m_ref, _parking_batch(), graph=True, warmup=1)
        opt = FlatAdam([p for p in m_ddp.parameters() if p.requires_grad], lr=1e-4, weight_decay=1e-4)

        def capture(fn, *a, **k):  # the table as the first (backward) capture found it
            if "key" not in saved:
                saved["key"] = opt._gkey
            return real_capture(fn, *a, **k)

        T.graphs.capture = capture
        s_ddp = (TrainStep(m_ddp, _parking_batch(), graph=True, warmup=1, ddp=True, bucket_mb=4.0,
                           overlap="captured", optimizer=opt) if hooks else
                 TrainStep(m_ddp, _parking_batch(), graph=True, warmup=1, optimizer=opt))
        T.graphs.capture = real_capture
        # round-4 check (verdict r3 item 8): the weights both modules carry into the capture,
        # i.e. after their eager warm-up step, against each other and the initial weights
        w0 = dict(_parking_module().named_parameters())
        wr, wd = dict(m_ref.named_parameters()), dict(m_ddp.named_parameters())
        n_ref_moved = sum(not torch.equal(wr[k], w0[k]) for k in w0 if wr[k].requires_grad)
        n_ddp_moved = sum(not torch.equal(wd[k], w0[k]) for k in w0 if wd[k].requires_grad)
        n_diff = sum(not torch.equal(wr[k], wd[k]) for k in w0 if wr[k].requires_grad)
        print(f"{tag}: after warm-up: ref moved {n_ref_moved}, hooked moved {n_ddp_moved}, "
              f"differ {n_diff} (of {sum(p.requires_grad for p in w0.values())}); hooked has-grad "
              f"mask sum {int(s_ddp.has_grad.sum()) if s_ddp.has_grad is not None else None}",
              flush=True)
        del w0
        if not hooks:  # harness check: two plain captured steps
            s_ref.g_bwd.replay()
            s_ddp.g_bwd.replay()
            torch.cuda.synchronize()
            pr = [p for p in m_ref.parameters() if p.requires_grad]
            pd_ = [p for p in m_ddp.parameters() if p.requires_grad]
            nbad = sum(not torch.equal(a.grad, b.grad) for a, b in zip(pr, pd_) if a.grad is not None)
            print(f"{tag}: two hook-free captured steps: {nbad} of {len(pr)} gradients differ", flush=True)
            return
        live = [p.grad.data_ptr() if p.grad is not None else 0 for p in opt.params]
        stale = list(saved["key"])
        moved = sum(a != b for a, b in zip(live, stale))
        if not reprepare:  # back to the warm-up addresses, as the round-2 replay had them
            opt._gtab.copy_(torch.tensor(stale, dtype=torch.int64))
        print(f"{tag}: {moved} / {len(live)} gradient addresses differ between the eager warm-up "
              f"and the capture", flush=True)
        s_ref.g_bwd.replay()
        s_ddp.g_bwd.replay()
        gref = torch.zeros_like(s_ddp.flat_grad)
        s_ref.opt.prepare()
        s_ref.opt.gather_grads(gref)
        torch.cuda.synchronize()
        names = [n for n, p in m_ddp.named_parameters() if p.requires_grad]
        pd = dict(m_ddp.named_parameters())
        bad_grad = bad_flat = 0
        first = None
        for i, (o, n) in enumerate(s_ddp.opt.spans):
            ref = gref[o:o + n]
            g = pd[names[i]].grad
            if g is None or not torch.equal(g.reshape(-1), ref):
                bad_grad += 1
                first = first or names[i]
            if not torch.equal(s_ddp.flat_grad[o:o + n], ref):
                bad_flat += 1
        lr, ld = float(s_ref.loss), float(s_ddp.loss)
        rel = []
        for i, (o, n) in enumerate(s_ddp.opt.spans):
            g = pd[names[i]].grad
            if g is not None:
                ref = gref[o:o + n]
                rel.append(((g.reshape(-1) - ref).norm() / ref.norm().clamp_min(1e-30)).item())
        rel.sort()
        print(f"{tag}: captured loss ref {lr:.6f} hooks {ld:.6f}; per-tensor rel-L2 of the "
              f"autograd gradients: median {rel[len(rel) // 2]:.3e} max {rel[-1]:.3e} "
              f"(last-computed tensors first: {[f'{r:.1e}' for r in rel[-3:]]})", flush=True)
        print(f"{tag}: wgrad_fork={wgrad_fork} reprepare={reprepare}: autograd .grad wrong "
              f"{bad_grad} / {len(names)}, gathered flat wrong {bad_flat} / {len(names)}, "
              f"buckets {len(s_ddp.buckets.buckets)}; first wrong: {first}", flush=True)
    finally:
        dist.all_reduce = real_ar
        T.GradBuckets.finish = real_finish
        T.graphs.capture = real_capture
        conv._OVERLAP[0] = True


# A reads freed memory through the stale table: on this stack it ends in an illegal-address
# fault of the replay (profiles/r03/ddp_diag/diag_capture_hooks_A.log), so it only runs when
# asked for; the default runs C (the fix).
VARIANTS = {"A": (True, False, True), "B": (False, False, True), "C": (True, True, True),
            "R": (True, True, False), "CN": (False, True, True)}
for tag in (sys.argv[1:] or ["R", "C"]):
    run(tag, *VARIANTS[tag])
dist.destroy_process_group()
print("done", flush=True)
