"""Depthwise conv kernel A/B on the C2 step's EfficientNet-B4 shapes (N = 32 camera images of
256 x 256): GPU time per e2ep_dwconv_fwd / _dgrad / _wgrad call (20 calls in one HIP graph),
and the step total weighted by how many layers have each shape, for each e2ep_tune setting
given ("key=value,..."; "" = defaults).

    python scripts/bench_dw.py [--tune '' '23=1' ...]"""
import argparse
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "e2e-parking-carla_amd"), ROOT, os.path.join(ROOT, "scripts")]
import torch  # noqa: E402

from bench_gemm import timed  # noqa: E402

# (C, H, K, stride, layers) of the reference's EfficientNet-B4 trunk up to reduction_4
# (model/cam_encoder.py), N = 8 samples x 4 cameras
SHAPES = [(48, 128, 3, 1, 1), (24, 128, 3, 1, 1), (144, 128, 3, 2, 1), (192, 64, 3, 1, 3),
          (192, 64, 5, 2, 1), (336, 32, 5, 1, 3), (336, 32, 3, 2, 1), (672, 16, 3, 1, 5),
          (672, 16, 5, 1, 1), (960, 16, 5, 1, 5)]
N = 32


def pads(H, K, st):
    """TF 'same' padding (left, right, top, bottom) as the reference's Conv2dStaticSamePadding."""
    out = (H + st - 1) // st
    tot = max((out - 1) * st + K - H, 0)
    return tot // 2, tot - tot // 2, tot // 2, tot - tot // 2


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--tune", nargs="+", default=[""])
    args = ap.parse_args()
    from e2ep_amd import _lib
    lib = _lib.load()
    base = {}
    for sv in args.tune:
        changed = []
        for kv in filter(None, sv.split(",")):
            k, v = (int(t) for t in kv.split("="))
            changed.append((k, lib.e2ep_tune(k, v)))
        tot = {"fwd": 0.0, "dgrad": 0.0, "wgrad": 0.0}
        print(f"== tune '{sv}'")
        for C, H, K, st, n in SHAPES:
            l, r, t, b = pads(H, K, st)
            P = (H + t + b - K) // st + 1
            x = torch.randn(N, C, H, H, device="cuda")
            w = torch.randn(C, 1, K, K, device="cuda")
            gy = torch.randn(N, C, P, P, device="cuda")
            y = torch.empty_like(gy)
            dx = torch.empty_like(x)
            dw = torch.empty_like(w)
            d = _lib.dims((N, C, H, H, K, P, P, st, t, l))
            ws = torch.empty(max(lib.e2ep_dwconv_wgrad_workspace(d), 4), dtype=torch.uint8,
                             device="cuda")
            s = _lib.stream

            def fwd():
                _lib.call("e2ep_dwconv_fwd", _lib.ptr(x), _lib.ptr(w), d, None, None, 0,
                          _lib.ptr(y), s())

            def dgr():
                _lib.call("e2ep_dwconv_dgrad", _lib.ptr(gy), _lib.ptr(w), d, _lib.ptr(dx), s(), 0)

            def wgr():
                _lib.call("e2ep_dwconv_wgrad", _lib.ptr(gy), _lib.ptr(x), d, None, None, 0,
                          _lib.ptr(ws), _lib.nbytes(ws), _lib.ptr(dw), s(), 0)

            us = {"fwd": timed(fwd, 20), "dgrad": timed(dgr, 20), "wgrad": timed(wgr, 20)}
            mb = 4 * N * C * (H * H + P * P) / 1e6
            key = (C, H, K, st)
            if sv == args.tune[0]:
                base[key] = us
            rel = " ".join(f"{k} {v:7.1f} us ({mb / v:5.2f} TB/s, x{base[key][k] / v:4.2f})"
                           for k, v in us.items())
            print(f"C{C:4d} H{H:4d} k{K} s{st} x{n}: {rel}", flush=True)
            for k in tot:
                tot[k] += n * us[k]
        print("step total us: " + " ".join(f"{k} {v:.0f}" for k, v in tot.items())
              + f" sum {sum(tot.values()):.0f}", flush=True)
        for k, v in changed:
            lib.e2ep_tune(k, v)


if __name__ == "__main__":
    main()
