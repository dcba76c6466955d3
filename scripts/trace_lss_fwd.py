"""Diagnostics: per-block start/end timestamps of k_lss_fwd (s_memrealtime, 100 MHz) at the
bench workload, to see block lifetimes, concurrency and the tail.  Writes gpurun_out/fwd_trace.npy."""
import ctypes
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "e2e-parking-carla_amd"), ROOT, os.path.join(ROOT, "scripts")]
from e2ep_amd import _lib  # noqa: E402

lib = _lib.load()
lib.e2ep_debug_fwd_trace.argtypes = [ctypes.c_void_p]
buf = torch.zeros(4 * 5000 * 4, dtype=torch.int64, device="cuda")
import bench_lss  # noqa: E402

sys.argv = [sys.argv[0], "--batch", "8", "--iters", "5"]
bench_lss.main()
lib.e2ep_debug_fwd_trace(ctypes.c_void_p(buf.data_ptr()))
bench_lss.main()
torch.cuda.synchronize()
t = buf.view(-1, 4).cpu().numpy()
t = t[t[:, 1] > 0]
os.makedirs(os.path.join(ROOT, "gpurun_out"), exist_ok=True)
np.save(os.path.join(ROOT, "gpurun_out", "fwd_trace.npy"), t)
t0 = t[:, 0].min()
st, en = (t[:, 0] - t0) * 10e-3, (t[:, 1] - t0) * 10e-3  # us
dur = en - st
print("blocks", len(t), "span us", en.max(), "mean dur", dur.mean(), "p50", np.median(dur), "max", dur.max())
pts = t[:, 3]
for lo, hi in ((0, 1), (1, 100), (100, 300), (300, 600), (600, 2000)):
    m = (pts >= lo) & (pts < hi)
    if m.any():
        print(f"pts [{lo},{hi}): n={m.sum()} mean dur {dur[m].mean():.2f} us, max {dur[m].max():.2f}")
hist = np.histogram(st, bins=20)[0]
print("start histogram (20 bins over span):", hist.tolist())
conc = [((st <= x) & (en > x)).sum() for x in np.linspace(0, en.max(), 20)]
print("blocks alive over time:", conc)
