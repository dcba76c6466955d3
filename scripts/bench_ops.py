"""Per-shape microbenchmark of the e2ep conv kernels against MIOpen (torch) on the conv
shapes one ParkingModel train step actually issues (recorded by running the model once).

    python scripts/bench_ops.py [--batch 8] [--top 30]
Prints, per shape: fwd / dgrad / wgrad time for e2ep and torch (ms), and FLOP rate."""
import argparse
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "e2e-parking-carla_amd"), ROOT]

import torch  # noqa: E402
import torch.nn.functional as F  # noqa: E402


def timeit(fn, reps=10):
    fn()
    torch.cuda.synchronize()
    s = torch.cuda.Event(enable_timing=True)
    e = torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(reps):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / reps


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=8)
    ap.add_argument("--top", type=int, default=40)
    args = ap.parse_args()
    from e2ep_amd import conv, synthetic
    from tool.config import default_cfg
    from trainer.pl_trainer import ParkingTrainingModule

    shapes = {}
    orig = conv.conv2d

    def rec(x, w, b=None, stride=(1, 1), pad=(0, 0, 0, 0), dilation=(1, 1), act=0, grad_channels=None):
        key = (tuple(x.shape), tuple(w.shape), tuple(stride), tuple(pad), tuple(dilation), b is not None)
        shapes[key] = shapes.get(key, 0) + 1
        return orig(x, w, b, stride, pad, dilation, act, grad_channels)

    conv.conv2d = rec
    mod = ParkingTrainingModule(default_cfg()).cuda().train()
    data = synthetic.synthetic_batch(args.batch, seed=0)
    mod.training_step(data).backward()
    conv.conv2d = orig
    rows = []
    for (xs, ws, st, pad, dil, hasb), cnt in shapes.items():
        x = torch.randn(xs, device="cuda", requires_grad=True)
        w = torch.randn(ws, device="cuda", requires_grad=True)
        y = orig(x, w, None, st, pad, dil)
        gy = torch.randn_like(y)
        N, Cin, H, W = xs
        Cout, _, R, S = ws
        flops = 2.0 * N * y.shape[2] * y.shape[3] * Cout * Cin * R * S
        t_f = timeit(lambda: orig(x, w, None, st, pad, dil))
        t_b = timeit(lambda: torch.autograd.grad(orig(x, w, None, st, pad, dil), (x, w), gy)) - t_f
        xp = F.pad(x.detach(), (pad[0], pad[1], pad[2], pad[3])).requires_grad_(True)
        t_tf = timeit(lambda: F.conv2d(xp, w, None, st, 0, dil))
        t_tb = timeit(lambda: torch.autograd.grad(F.conv2d(xp, w, None, st, 0, dil), (xp, w), gy)) - t_tf
        rows.append((cnt * (t_f + t_b), cnt, xs, ws, st, dil, t_f, t_b, t_tf, t_tb, flops))
    rows.sort(key=lambda r: -r[0])
    tot_e = sum(r[1] * (r[6] + r[7]) for r in rows)
    tot_t = sum(r[1] * (r[8] + r[9]) for r in rows)
    print(f"total per step: e2ep {tot_e:.2f} ms   torch/MIOpen {tot_t:.2f} ms   ({len(rows)} shapes)")
    print(f"{'x':>20} {'w':>18} st dil  n | e2ep fwd  bwd (TF/s) | torch fwd  bwd")
    for r in rows[:args.top]:
        _, cnt, xs, ws, st, dil, tf, tb, ttf, ttb, fl = r
        print(f"{str(xs):>20} {str(ws):>18} {st[0]} {dil[0]:>3} {cnt:2d} | {tf:7.3f} {tb:7.3f} ({fl / tf / 1e9:5.1f}) | {ttf:7.3f} {ttb:7.3f}")


if __name__ == "__main__":
    main()
