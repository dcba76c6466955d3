"""Diagnose the RCCL world-1 bucketed all-reduce path of TrainStep (eager vs captured)."""
import os
import socket
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "e2e-parking-carla_amd"), ROOT, os.path.join(ROOT, "tests")]
import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402

from test_ddp_gpu import _parking_batch, _parking_module, _flat_params  # noqa: E402
from e2ep_amd.train import TrainStep  # noqa: E402


def port():
    with socket.socket() as so:
        so.bind(("127.0.0.1", 0))
        return so.getsockname()[1]


os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port()))
dist.init_process_group("nccl", rank=0, world_size=1, device_id=torch.device("cuda", 0))
for graph in (False, True):
    m_ref, m_ddp = _parking_module(), _parking_module()
    s_ref = TrainStep(m_ref, _parking_batch(), graph=graph, warmup=1)
    s_ddp = TrainStep(m_ddp, _parking_batch(), graph=graph, warmup=1, ddp=True, bucket_mb=4.0)
    if not graph:
        s_ref(), s_ddp()
    print("graph", graph, "after warm-up: params equal", torch.equal(_flat_params(m_ref), _flat_params(m_ddp)),
          flush=True)
    for it in range(3):
        l_ref, l_ddp = float(s_ref()), float(s_ddp())
        # gradients of this step: ref's per-tensor .grad vs ddp's flat buffer
        gref = torch.zeros_like(s_ddp.flat_grad)
        s_ref.opt.prepare()
        s_ref.opt.gather_grads(gref)
        torch.cuda.synchronize()
        d = (gref - s_ddp.flat_grad).abs().max().item()
        print(f"graph {graph} step {it}: loss ref {l_ref:.6f} ddp {l_ddp:.6f}; max|grad ref - flat ddp| {d:.3e}; "
              f"params equal {torch.equal(_flat_params(m_ref), _flat_params(m_ddp))}", flush=True)
dist.destroy_process_group()
