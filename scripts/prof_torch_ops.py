"""Diagnostics: which PyTorch ops (not e2ep kernels) run in one eager train step, how often,
and from which model source lines.  python scripts/prof_torch_ops.py > gpurun_out/torch_ops.txt"""
import collections
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "e2e-parking-carla_amd"), ROOT]
import torch  # noqa: E402
from torch.profiler import ProfilerActivity, profile  # noqa: E402

from e2ep_amd import synthetic  # noqa: E402
from tool.config import default_cfg  # noqa: E402
from trainer.pl_trainer import ParkingTrainingModule  # noqa: E402

dev = torch.device("cuda")
torch.manual_seed(0)
mod = ParkingTrainingModule(default_cfg()).to(dev).train()
data = {k: (v if k in ("intrinsics", "extrinsics") else v.to(dev)) for k, v in
        synthetic.synthetic_batch(8, seed=0).items()}
for _ in range(2):
    mod.training_step(data, 0).backward()
torch.cuda.synchronize()
with profile(activities=[ProfilerActivity.CPU], with_stack=True, record_shapes=False) as prof:
    mod.zero_grad(set_to_none=True)
    mod.training_step(data, 0).backward()
    torch.cuda.synchronize()
skip = ("aten::empty", "aten::view", "aten::as_strided", "aten::reshape", "aten::detach",
        "aten::t", "aten::transpose", "aten::expand", "aten::_unsafe_view", "aten::slice",
        "aten::select", "aten::unsqueeze", "aten::squeeze", "aten::permute", "aten::alias",
        "aten::empty_like", "aten::empty_strided", "aten::lift_fresh", "aten::resolve_conj",
        "aten::resolve_neg", "aten::item", "aten::_local_scalar_dense", "aten::is_nonzero")
cnt = collections.Counter()
sites = collections.defaultdict(collections.Counter)
for ev in prof.events():
    if not ev.name.startswith("aten::") or ev.name in skip:
        continue
    cnt[ev.name] += 1
    st = [f for f in (ev.stack or []) if any(k in f for k in ("model/", "e2ep_amd/", "loss/", "trainer/"))]
    sites[ev.name][st[0] if st else "(autograd engine / torch internals)"] += 1
ex = [ev for ev in prof.events() if ev.name == "aten::add_"][:2]
for ev in ex:
    print("example stack:", ev.stack[:8])
for name, n in cnt.most_common(40):
    print(f"{n:5d} {name}")
    for site, m in sites[name].most_common(4):
        print(f"        {m:4d} {site}")
