"""Diagnostics: run one conv shape's forward / data-gradient / weight-gradient kernels
repeatedly (for rocprofv3 --pmc passes and kernel-trace timing).

    python scripts/conv_pmc.py <shape> [fwd|dgrad|wgrad|all] [reps]
(E2EP_PRECISION=bf16 for the C3 kernels)"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "e2e-parking-carla_amd"), ROOT]
import torch  # noqa: E402

from e2ep_amd import conv  # noqa: E402

SHAPES = {"stem": (8, 65, 256, 256, 64, 7, 7, 128, 128, 2, 2, 3, 3, 1, 1),
          "stem64": (8, 64, 256, 256, 64, 7, 7, 128, 128, 2, 2, 3, 3, 1, 1),
          "seg": (8, 64, 200, 200, 64, 3, 3, 200, 200, 1, 1, 1, 1, 1, 1),
          "l1": (8, 64, 64, 64, 64, 3, 3, 64, 64, 1, 1, 1, 1, 1, 1),
          "proj960": (32, 960, 16, 16, 160, 1, 1, 16, 16, 1, 1, 0, 0, 1, 1),
          "exp160": (32, 160, 16, 16, 960, 1, 1, 16, 16, 1, 1, 0, 0, 1, 1),
          "bev256": (8, 256, 16, 16, 256, 3, 3, 16, 16, 1, 1, 1, 1, 1, 1),
          "up216": (32, 216, 32, 32, 64, 3, 3, 32, 32, 1, 1, 1, 1, 1, 1),
          "exp112": (32, 112, 16, 16, 672, 1, 1, 16, 16, 1, 1, 0, 0, 1, 1)}
# data-gradient rows the product computes (bev_stem.py: the target-point plane, input channel
# 64 of the stem, is a constant and gets no gradient; round 3's PMC ran 65 rows: two 64-row
# tiles, twice the MFMA work of the product's launch)
GRAD_CHANNELS = {"stem": 64}


def main():
    which = sys.argv[1] if len(sys.argv) > 1 else "seg"
    kind = sys.argv[2] if len(sys.argv) > 2 else "all"
    reps = int(sys.argv[3]) if len(sys.argv) > 3 else 10
    d = SHAPES[which]
    if os.environ.get("E2EP_PRECISION"):  # fp32 (default) / bf16 / fp16 operands
        from e2ep_amd import precision
        precision.set(os.environ["E2EP_PRECISION"])
    if os.environ.get("E2EP_GEMM_VARIANT"):
        from e2ep_amd import _lib
        _lib.call_raw("e2ep_conv_gemm_variant", int(os.environ["E2EP_GEMM_VARIANT"]))
    N, Cin, H, W, Cout, R, S, P, Q = d[:9]
    g = torch.Generator(device="cuda").manual_seed(0)
    x = torch.randn(N, Cin, H, W, device="cuda", generator=g)
    wt = conv.tap_major(torch.randn(Cout, Cin, R, S, device="cuda", generator=g) * 0.05)
    gy = torch.randn(N, Cout, P, Q, device="cuda", generator=g)
    y = torch.empty(N, Cout, P, Q, device="cuda")
    gc = GRAD_CHANNELS.get(which, Cin)
    dx = torch.empty(N, gc, H, W, device="cuda")
    dw = torch.empty(Cout, Cin, R, S, device="cuda")
    for _ in range(reps):
        if kind in ("fwd", "all"):
            conv.conv_fwd(x, wt, None, d, 0, y, w_layout=1)
        if kind in ("dgrad", "all"):
            conv.conv_dgrad(gy, wt, d, gc, dx, w_layout=1)
        if kind in ("wgrad", "all"):
            conv.conv_wgrad(gy, x, d, dw)
    torch.cuda.synchronize()


if __name__ == "__main__":
    main()
