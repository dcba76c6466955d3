"""Does a side-stream fork/join inside a captured backward corrupt the captured step on this
ROCm stack?  Capture TrainStep's backward with hooks that only fork an empty side stream off
the capture stream (event record + wait) and join it after backward; no collective, no
gather.  Compare the replayed gradients with a capture without hooks."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "e2e-parking-carla_amd"), ROOT, os.path.join(ROOT, "tests")]
import torch  # noqa: E402

from test_ddp_gpu import _parking_batch, _parking_module  # noqa: E402
from e2ep_amd.train import TrainStep  # noqa: E402


class ForkOnly:
    def __init__(self, params, work):
        self.side = torch.cuda.Stream()
        self.active = False
        self.work = work
        self.n = 0
        for p in params:
            p.register_post_accumulate_grad_hook(self.hook)

    def hook(self, _p):
        if not self.active:
            return
        self.n += 1
        if self.n % 20:
            return
        ev = torch.cuda.Event()
        ev.record(self.main)
        self.side.wait_event(ev)
        if self.work:
            with torch.cuda.stream(self.side):
                self.buf.add_(1.0)


for work in (False, True):
    m_ref, m_f = _parking_module(), _parking_module()
    s_ref = TrainStep(m_ref, _parking_batch(), graph=True, warmup=1)
    f = ForkOnly([p for p in m_f.parameters() if p.requires_grad], work)
    f.buf = torch.zeros(16, device="cuda")
    orig = TrainStep._fwd_bwd

    def fwd_bwd(self, f=f):
        f.active, f.n, f.main = True, 0, torch.cuda.current_stream()
        loss = orig(self)
        f.main.wait_stream(f.side)
        f.active = False
        return loss

    TrainStep._fwd_bwd = fwd_bwd
    s_f = TrainStep(m_f, _parking_batch(), graph=True, warmup=1)
    TrainStep._fwd_bwd = orig
    s_ref.g_bwd.replay()
    s_f.g_bwd.replay()
    torch.cuda.synchronize()
    pr = dict(m_ref.named_parameters())
    bad = [n for n, p in m_f.named_parameters() if p.grad is not None and not torch.equal(p.grad, pr[n].grad)]
    print(f"fork-only (side work={work}): {len(bad)} gradients differ; first: {bad[:3]}", flush=True)
