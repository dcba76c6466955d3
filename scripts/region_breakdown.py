"""Per-region, per-shape timing of the C2 train step (B=8): every e2ep op region of 3 eager
fwd+bwd passes bracketed by HIP events (E2EP_TIMING_DETAIL=1).  Prints the totals per kind
and the top entries with the activation size (MB of the region's main tensor) and how many
passes over it the measured time corresponds to at 5 TB/s."""
import os
import sys
from collections import defaultdict

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "e2e-parking-carla_amd"), ROOT]
os.environ["E2EP_TIMING_DETAIL"] = "1"
import torch  # noqa: E402


def main():
    from e2ep_amd import synthetic, timing
    from e2ep_amd.train import TrainStep
    from tool.config import default_cfg
    from trainer.pl_trainer import ParkingTrainingModule
    torch.manual_seed(0)
    mod = ParkingTrainingModule(default_cfg()).cuda().train()
    for p in mod.parking_model.bev_encoder.layer4.parameters():
        p.requires_grad_(False)
    d = synthetic.synthetic_batch(8, seed=0)
    d = {k: (v if k in ("intrinsics", "extrinsics") else v.cuda()) for k, v in d.items()}
    step = TrainStep(mod, d, graph=False)
    step()
    step()
    timing.reset()
    timing.enable(True)
    n = 3
    for _ in range(n):
        step._fwd_bwd()
    timing.enable(False)
    summ = timing.summary()
    kinds = defaultdict(float)
    rows = []
    for k, (cnt, mean, tot) in summ.items():
        kind = k.split("(")[0]
        kinds[kind] += tot / n
        mb = 0.0
        if "(" in k:
            shape = eval(k[len(kind):k.index(")") + 1])
            numel = 1
            for v in shape:
                numel *= v
            mb = numel * 4 / 1e6
        rows.append((tot / n, k, cnt / n, mean * 1e3, mb))
    print("per kind (ms/step):")
    for kind, t in sorted(kinds.items(), key=lambda kv: -kv[1]):
        print(f"  {kind:14s} {t:7.3f}")
    rows.sort(key=lambda r: -r[0])
    print(f"{'ms/step':>8s} {'n':>4s} {'us':>8s} {'MB':>8s} {'passes@5TB/s':>12s}  region")
    for t, k, cnt, us, mb in rows[:70]:
        passes = (us * 1e-6 * 5e12) / (mb * 1e6) if mb else 0.0
        print(f"{t:8.3f} {cnt:4.0f} {us:8.1f} {mb:8.1f} {passes:12.1f}  {k}")


if __name__ == "__main__":
    main()
