"""Microbenchmark of the lift-splat kernels (k_lss_fwd / k_lss_bwd) at the bench workload.

    python scripts/bench_lss.py [--batch 8] [--iters 50] [--cams 4 --image 256]
Times each kernel with HIP events on the launch stream (median of --iters launches) and
prints algorithmic GB/s (SURVEY.md §8d byte counts)."""
import argparse
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "e2e-parking-carla_amd"), ROOT]
import torch  # noqa: E402

from e2ep_amd import _lib, lss, synthetic  # noqa: E402
from model.bev_model import BevModel  # noqa: E402
from tool.config import default_cfg  # noqa: E402


def timeit(fn, iters):
    fn()
    torch.cuda.synchronize()
    ts = []
    for _ in range(iters):
        s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        s.record()
        fn()
        e.record()
        torch.cuda.synchronize()
        ts.append(s.elapsed_time(e))
    ts.sort()
    return ts[len(ts) // 2]


def timeit_b2b(fn, iters):
    """Mean of `iters` back-to-back launches between two events (launch gaps amortised)."""
    fn()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(iters):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / iters


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=8)
    ap.add_argument("--iters", type=int, default=50)
    ap.add_argument("--cams", type=int, default=4)
    ap.add_argument("--image", type=int, default=256)
    ap.add_argument("--fwd-variants", type=lambda t: [int(x) for x in t.split(",")], default=[1])
    a = ap.parse_args()
    dev = torch.device("cuda")
    cfg = default_cfg()
    if a.image != 256:
        cfg.final_dim = (a.image, a.image)
    bm = BevModel(cfg).to(dev)
    K, E = synthetic.rig(a.cams, a.image, *((512, 512) if a.image == 512 else ()))
    K = K.unsqueeze(0).expand(a.batch, *K.shape).contiguous()
    E = E.unsqueeze(0).expand(a.batch, *E.shape).contiguous()
    plan = bm.plan(K, E, dev)
    B, N, D, h, w, C = plan.B, plan.N, plan.D, plan.h, plan.w, 64
    hw, XY = h * w, plan.XYZ
    g = torch.Generator(device="cpu").manual_seed(0)
    prob = torch.rand(B * N, D, h, w, generator=g).to(dev)
    featT = torch.randn(B * N, hw, C, generator=g).to(dev)
    bev = torch.empty(B, C, plan.X, plan.Y, device=dev)
    gT = torch.randn(B, XY, C, generator=g).to(dev)
    gp, gf = torch.empty_like(prob), torch.empty(B * N, C, h, w, device=dev)

    def fwd():
        _lib.call("e2ep_lss_fwd", _lib.ptr(prob), _lib.ptr(featT), _lib.ptr(plan.offsets),
                  _lib.ptr(plan.order), None if os.environ.get("E2EP_NO_TILES") else _lib.ptr(plan.tiles), B, N, D, hw, C, XY, _lib.ptr(bev), C * XY, _lib.stream())

    def bwd():
        _lib.call("e2ep_lss_bwd", _lib.ptr(gT), _lib.ptr(prob), _lib.ptr(featT),
                  _lib.ptr(plan.pillar), B, N, D, hw, C, XY, _lib.ptr(gp), _lib.ptr(gf), _lib.stream())

    fb = 4 * B * (N * C * hw + N * D * hw + C * XY)
    bb = 4 * B * (C * XY + 2 * N * C * hw + 2 * N * D * hw)
    ref = None
    for v in a.fwd_variants:  # e2ep_tune key 32: the forward's groups x rows in flight
        prev = _lib.load().e2ep_tune(32, v)
        fwd()
        torch.cuda.synchronize()
        if ref is None:
            ref = bev.clone()
        same = torch.equal(bev, ref)  # every variant sums each pillar in the same order
        t1, t2 = timeit(fwd, a.iters), timeit_b2b(fwd, a.iters)
        print(f"lss_fwd[variant {v}] B={B} N={N} {a.image}^2: single {t1 * 1e3:.1f} us "
              f"({fb / t1 / 1e6:.0f} GB/s), back-to-back {t2 * 1e3:.1f} us ({fb / t2 / 1e6:.0f} GB/s); "
              f"{fb / 1e6:.1f} MB algorithmic; bitwise equal to variant {a.fwd_variants[0]}: {same}")
        _lib.load().e2ep_tune(32, prev)
    t1, t2 = timeit(bwd, a.iters), timeit_b2b(bwd, a.iters)
    print(f"lss_bwd B={B} N={N} {a.image}^2: single {t1 * 1e3:.1f} us ({bb / t1 / 1e6:.0f} GB/s), "
          f"back-to-back {t2 * 1e3:.1f} us ({bb / t2 / 1e6:.0f} GB/s); {bb / 1e6:.1f} MB algorithmic")


if __name__ == "__main__":
    main()
