"""Time the forward / data-gradient GEMM variants (e2ep_conv_gemm_variant 1 vs 2) on the
hot conv shapes: 20 back-to-back launches between HIP events per (shape, kind, variant)."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "e2e-parking-carla_amd"), ROOT, os.path.join(ROOT, "scripts")]
import torch  # noqa: E402

from conv_pmc import SHAPES  # noqa: E402
from e2ep_amd import _lib, conv  # noqa: E402


def timeit(fn, reps=20):
    for _ in range(3):
        fn()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    torch.cuda.synchronize()
    s.record()
    for _ in range(reps):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / reps


def main():
    names = sys.argv[1:] or list(SHAPES)
    for name in names:
        d = SHAPES[name]
        N, Cin, H, W, Cout, R, S, P, Q = d[:9]
        g = torch.Generator(device="cuda").manual_seed(0)
        x = torch.randn(N, Cin, H, W, device="cuda", generator=g)
        wt = conv.tap_major(torch.randn(Cout, Cin, R, S, device="cuda", generator=g) * 0.05)
        gy = torch.randn(N, Cout, P, Q, device="cuda", generator=g)
        y = torch.empty(N, Cout, P, Q, device="cuda")
        dx = torch.empty(N, Cin, H, W, device="cuda")
        fl = conv.conv_flops(d)
        res = {}
        for v in (1, 2, 3):
            _lib.call_raw("e2ep_conv_gemm_variant", v)
            tf = timeit(lambda: conv.conv_fwd(x, wt, None, d, 0, y, w_layout=1))
            y1 = y.clone()
            tg = timeit(lambda: conv.conv_dgrad(gy, wt, d, Cin, dx, w_layout=1))
            dw = torch.empty(Cout, Cin, R, S, device="cuda")
            tw = timeit(lambda: conv.conv_wgrad(gy, x, d, dw))
            res[v] = (tf, tg, y1, dx.clone(), tw, dw.clone())
        _lib.call_raw("e2ep_conv_gemm_variant", 0)
        y1, d1, w1 = res[1][2], res[1][3], res[1][5]
        line = f"{name:8s}"
        for v in (1, 2, 3):
            f, gg, yv, dv, tw, wv = res[v]
            ey = float((yv - y1).norm() / y1.norm())
            ed = float((dv - d1).norm() / d1.norm())
            ew = float((wv - w1).norm() / w1.norm())
            line += (f" | v{v} fwd {f * 1e3:6.1f} us {fl / f / 1e9:5.1f} TF/s dgrad {gg * 1e3:6.1f} us "
                     f"{fl / gg / 1e9:5.1f} wgrad {tw * 1e3:6.1f} us {fl / tw / 1e9:5.1f} "
                     f"(d {ey:.0e} {ed:.0e} {ew:.0e})")
        print(line, flush=True)


if __name__ == "__main__":
    main()
