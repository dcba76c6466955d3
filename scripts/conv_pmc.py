"""Diagnostics: run a few conv shapes repeatedly (for rocprofv3 --pmc passes)."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "e2e-parking-carla_amd"), ROOT]
import torch  # noqa: E402

from e2ep_amd import conv  # noqa: E402

SHAPES = {"seg": (8, 64, 200, 200, 64, 3, 3, 200, 200, 1, 1, 1, 1, 1, 1),
          "proj960": (32, 960, 16, 16, 160, 1, 1, 16, 16, 1, 1, 0, 0, 1, 1),
          "bev256": (8, 256, 16, 16, 256, 3, 3, 16, 16, 1, 1, 1, 1, 1, 1)}
which = sys.argv[1] if len(sys.argv) > 1 else "seg"
d = SHAPES[which]
N, Cin, H, W, Cout, R, S, P, Q = d[:9]
x = torch.randn(N, Cin, H, W, device="cuda")
w = conv.tap_major(torch.randn(Cout, Cin, R, S, device="cuda"))
y = torch.empty(N, Cout, P, Q, device="cuda")
for _ in range(10):
    conv.conv_fwd(x, w, None, d, 0, y, w_layout=1)
torch.cuda.synchronize()
