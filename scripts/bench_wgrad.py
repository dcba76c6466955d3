"""Weight-gradient kernel A/B on the C2 step's conv shapes: GPU time per e2ep_conv_wgrad call
(kernel + split reduction), 20 calls captured in one HIP graph, for every pixel K-step
(e2ep_conv_wgrad_kstep) and precision given.

    python scripts/bench_wgrad.py [--ksteps 16 32] [--precisions fp32 bf16]"""
import argparse
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "e2e-parking-carla_amd"), ROOT]
import torch  # noqa: E402

from bench_gemm import timed  # noqa: E402  (same directory)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--ksteps", type=int, nargs="+", default=[16, 32])
    ap.add_argument("--precisions", nargs="+", default=["fp32"])
    ap.add_argument("--top", type=int, default=25)
    args = ap.parse_args()
    from e2ep_amd import _lib, conv, precision
    with open(os.path.join(ROOT, "scripts", "conv_shapes.json")) as f:
        shapes = json.load(f)
    rows = []
    for sh in shapes:
        d = sh["dims"]
        N, Cin, H, W, Cout, R, S, P, Q = d[:9]
        if R * S == 1:  # 1x1 weight gradients mostly take the LDS-free kernel
            continue
        x = torch.randn(N, Cin, H, W, device="cuda")
        gy = torch.randn(N, Cout, P, Q, device="cuda")
        dw = torch.empty(Cout, Cin, R, S, device="cuda")
        res = {}
        for prec in args.precisions:
            for kb in args.ksteps:
                old = _lib.call_raw("e2ep_conv_wgrad_kstep", kb)
                with precision.use(prec):
                    res[f"{prec}/k{kb}"] = timed(lambda: conv.conv_wgrad(gy, x, tuple(d), dw), 20)
                _lib.call_raw("e2ep_conv_wgrad_kstep", old)
        rows.append((sh["count"], d, res))
    rows.sort(key=lambda r: -r[0] * max(r[2].values()))
    tot = {}
    for cnt, d, res in rows[:args.top]:
        print(f"{cnt:2d}x {str(d):60s} " + "  ".join(f"{k} {v:7.1f}" for k, v in res.items()), flush=True)
    for cnt, d, res in rows:
        for k, v in res.items():
            tot[k] = tot.get(k, 0.0) + cnt * v
    print("per step (ms):", {k: round(v / 1e3, 3) for k, v in tot.items()})


if __name__ == "__main__":
    main()
