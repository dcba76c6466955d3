"""Narrow down the captured bucket all-reduce: pure RCCL capture, side-stream capture, and
TrainStep with the collective stubbed out."""
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
from e2ep_amd import graphs  # noqa: E402

# A: all_reduce on the capture stream
t = torch.ones(1000, device="cuda")
dist.all_reduce(t)
torch.cuda.synchronize()
g = torch.cuda.CUDAGraph()
with torch.cuda.graph(g):
    t.mul_(2.0)
    dist.all_reduce(t)
for _ in range(3):
    g.replay()
torch.cuda.synchronize()
print("A capture-stream all_reduce: t[0] =", t[0].item(), "(want 8)", flush=True)

# B: async all_reduce forked onto a side stream, joined by wait()
t2 = torch.ones(1000, device="cuda")
side = torch.cuda.Stream()
g2 = torch.cuda.CUDAGraph()
with torch.cuda.graph(g2):
    t2.mul_(2.0)
    ev = torch.cuda.Event()
    ev.record(torch.cuda.current_stream())
    side.wait_event(ev)
    with torch.cuda.stream(side):
        print("  side capturing:", torch.cuda.is_current_stream_capturing(), flush=True)
        t2.add_(1.0)
        w = dist.all_reduce(t2, async_op=True)
    w.wait()
    torch.cuda.current_stream().wait_stream(side)
    t2.mul_(10.0)
for _ in range(2):
    g2.replay()
torch.cuda.synchronize()
print("B side-stream async all_reduce: t2[0] =", t2[0].item(), "(want ((1*2+1)*10*2+1)*10 = 610)", flush=True)

# B': same with the e2ep memset repair
t3 = torch.ones(1000, device="cuda")


def body():
    t3.mul_(2.0)
    ev = torch.cuda.Event()
    ev.record(torch.cuda.current_stream())
    side.wait_event(ev)
    with torch.cuda.stream(side):
        t3.add_(1.0)
        w = dist.all_reduce(t3, async_op=True)
    w.wait()
    torch.cuda.current_stream().wait_stream(side)
    t3.mul_(10.0)


g3, _, nm = graphs.capture(body)
for _ in range(2):
    g3.replay()
torch.cuda.synchronize()
print("B' repaired graph:", t3[0].item(), "(want 610), memsets replaced", nm, flush=True)

# C: TrainStep with the collective stubbed out (gather only)
from test_ddp_gpu import _parking_batch, _parking_module  # noqa: E402
from e2ep_amd.train import TrainStep  # noqa: E402


class _Done:
    def wait(self):
        pass


import e2ep_amd.train as T  # noqa: E402
_orig_launch = T.GradBuckets._launch


def _spy(self, b):
    if b in (0,) and not getattr(self, "_spied", False):
        cur = torch.cuda.current_stream()
        print(f"   bucket {b}: hook stream {cur.cuda_stream:#x} main {self.main.cuda_stream:#x} "
              f"capturing(main)={self.capturing} capturing(hook)={torch.cuda.is_current_stream_capturing()}",
              flush=True)
    return _orig_launch(self, b)


T.GradBuckets._launch = _spy
real = dist.all_reduce
for stub in (True, False):
    if stub:
        dist.all_reduce = lambda t, async_op=False, **k: _Done()
    else:
        dist.all_reduce = real
    m_ref, m_ddp = _parking_module(), _parking_module()
    s_ref = TrainStep(m_ref, _parking_batch(), graph=True, warmup=1)
    s_ddp = TrainStep(m_ddp, _parking_batch(), graph=True, warmup=1, ddp=True, bucket_mb=4.0)
    s_ref.g_bwd.replay()
    s_ddp.g_bwd.replay()
    gref = torch.zeros_like(s_ddp.flat_grad)
    s_ref.opt.gather_grads(gref)
    torch.cuda.synchronize()
    bad = torch.isnan(s_ddp.flat_grad).sum().item()
    d = (gref - s_ddp.flat_grad).abs().max().item()
    print(f"C stub={stub}: max|diff| {d:.3e}, nan count {bad}, n buckets {len(s_ddp.buckets.buckets)}",
          flush=True)
    # which buckets are wrong
    names = [n for n, p in m_ddp.named_parameters() if p.requires_grad]
    nbad = 0
    for i, (o, n) in enumerate(s_ddp.opt.spans):
        a, b = gref[o:o + n], s_ddp.flat_grad[o:o + n]
        dd = (a - b).abs().max().item()
        if dd != 0.0:
            nbad += 1
            if nbad <= 12 or i < 3:
                pg = dict(m_ddp.named_parameters())[names[i]].grad
                print(f"   param {i} {names[i]} n={n} maxdiff {dd:.3e} |ref| {a.abs().max().item():.3e} "
                      f"|flat| {b.abs().max().item():.3e} ddp.grad==ref {torch.equal(pg.reshape(-1), a)} "
                      f"flat==ddp.grad {torch.equal(pg.reshape(-1), b)} gtab ok "
                      f"{int(s_ddp.opt._gtab[i]) == pg.data_ptr()}", flush=True)
    print("   params wrong:", nbad, "of", len(names), flush=True)
dist.all_reduce = real
dist.destroy_process_group()
