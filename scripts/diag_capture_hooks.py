"""Diagnostic (verdict r3, item 8): the cause of round 3's unexplained variant CN.

Round 3 ran the round-2 data-parallel graph design (post-accumulate-grad hooks gathering and
all-reducing buckets INSIDE the captured backward) with the all-reduce stubbed out and the
gradient table re-pointed, and still saw the hooked capture diverge from a hook-free one
(captured loss 13.286 vs 11.209, 530 of 530 gradients wrong; profiles/r03/ddp_diag/
diag_capture_hooks_CN.log).  That diagnostic patched GradBuckets.finish with a round-2 copy
that, unlike the real one, never refreshed the has-gradient mask (`opt.has_grad(self.has)`),
so the hooked module's eager warm-up step called FlatAdam.step(flat, has_grad=<all zeros>)
and stepped no parameter: the two modules entered the capture with different weights
(initial vs after one Adam step), and everything downstream differed for that reason alone.

This script shows it without any capture (the warm-up step is an ordinary eager step; the
captured path itself was removed from TrainStep in round 4): one eager hooked data-parallel
step with that patched finish, and one with the real finish, each against a hook-free step
of the same module, printing how many parameters moved and how many differ.  Expected:
patched finish -> the hooked module moves 0 of 530 parameters; real finish -> 530, and the
same values as the hook-free step (0 differ).  World-1 RCCL, all-reduce stubbed."""
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
from e2ep_amd.train import TrainStep  # noqa: E402


class _Done:
    def wait(self):
        pass


real_ar = dist.all_reduce
real_finish = T.GradBuckets.finish


def finish_round3_diag(self):
    """GradBuckets.finish as round 3's diagnostic patched it: no has-gradient mask update."""
    while self.next < len(self.buckets):
        self._launch(self.next)
        self.next += 1
    for w in self.works:
        w.wait()
    self.main.wait_stream(self.comm)
    if not self.capturing:
        self.opt.prepare()
    self.works = []
    self.active = False


def run(tag, finish):
    T.GradBuckets.finish = finish
    dist.all_reduce = lambda t, async_op=False, **k: _Done()
    try:
        w0 = {k: v.detach().clone() for k, v in _parking_module().named_parameters()}
        m_ref, m_hook = _parking_module(), _parking_module()
        s_ref = TrainStep(m_ref, _parking_batch(), graph=False)
        s_hook = TrainStep(m_hook, _parking_batch(), graph=False, ddp=True, overlap=True,
                           bucket_mb=4.0)
        assert s_hook.buckets is not None
        l_ref, l_hook = float(s_ref()), float(s_hook())
        torch.cuda.synchronize()
        wr, wh = dict(m_ref.named_parameters()), dict(m_hook.named_parameters())
        keys = [k for k in w0 if wr[k].requires_grad]
        moved_r = sum(not torch.equal(wr[k], w0[k]) for k in keys)
        moved_h = sum(not torch.equal(wh[k], w0[k]) for k in keys)
        differ = sum(not torch.equal(wr[k], wh[k]) for k in keys)
        print(f"{tag}: step loss ref {l_ref:.6f} hooked {l_hook:.6f}; parameters moved: ref "
              f"{moved_r}, hooked {moved_h}; differ {differ} of {len(keys)}; has-grad mask sum "
              f"{int(s_hook.has_grad.sum())}", flush=True)
    finally:
        dist.all_reduce = real_ar
        T.GradBuckets.finish = real_finish


run("round3-diag finish (no has-grad mask)", finish_round3_diag)
run("real finish", real_finish)
dist.destroy_process_group()
print("done", flush=True)
