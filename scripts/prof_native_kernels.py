"""Diagnostics: every PyTorch-native (at::native) GPU kernel one eager TrainStep (the bench's
step: fwd + 3 losses + bwd + Adam, B = 8) launches, with the aten op that launched it and the
model / product source line of that op.

    python scripts/prof_native_kernels.py [--precision bf16] > gpurun_out/native_kernels.txt"""
import argparse
import collections
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "e2e-parking-carla_amd"), ROOT]
import torch  # noqa: E402
from torch.profiler import ProfilerActivity, profile  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--precision", default="fp32")
    a = ap.parse_args()
    from bench import device_batch
    from e2ep_amd import precision, synthetic
    from e2ep_amd.train import TrainStep
    from tool.config import default_cfg
    from trainer.pl_trainer import ParkingTrainingModule

    precision.set(a.precision)
    dev = torch.device("cuda")
    torch.manual_seed(1234)
    mod = ParkingTrainingModule(default_cfg()).to(dev).train()
    for p in mod.parking_model.bev_encoder.layer4.parameters():
        p.requires_grad_(False)
    data = device_batch(synthetic.synthetic_batch(8, seed=0), dev)
    step = TrainStep(mod, data, lr=mod.cfg.learning_rate, weight_decay=mod.cfg.weight_decay,
                     world=1, graph=False, warmup=1)
    for _ in range(2):
        step()
    torch.cuda.synchronize()
    with profile(activities=[ProfilerActivity.CPU, ProfilerActivity.CUDA], with_stack=True) as prof:
        step()
        torch.cuda.synchronize()
    evs = prof.events()
    by_id = {ev.id: ev for ev in evs}
    keys = ("model/", "e2ep_amd/", "loss/", "trainer/", "bench.py")
    rows = collections.Counter()
    for ev in evs:
        kern = getattr(ev, "kernels", None) or []
        for k in kern:
            if "at::native" not in k.name and "elementwise" not in k.name:
                continue
            # the innermost aten op that launched it and the first product frame up its parents
            op = ev
            site = None
            p = ev
            while p is not None and site is None:
                st = [f for f in (p.stack or []) if any(s in f for s in keys)]
                if st:
                    site = st[0]
                p = getattr(p, "cpu_parent", None)
            kn = k.name.split("<")[0] + "<" + k.name.split("<")[1][:90] if "<" in k.name else k.name
            rows[(op.name, kn, site or "(autograd engine)")] += 1
    for (op, kn, site), n in sorted(rows.items(), key=lambda r: -r[1]):
        print(f"{n:4d}  {op:32s} {site}\n        {kn}")
    print(f"total native kernel launches: {sum(rows.values())}")


if __name__ == "__main__":
    main()
