"""Diagnostics: GPU time of the PyTorch (non-e2ep) ops of one eager train step, by aten op
and by input shapes.  python scripts/prof_torch_time.py > gpurun_out/torch_time.txt"""
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
with profile(activities=[ProfilerActivity.CPU, ProfilerActivity.CUDA], record_shapes=True) as prof:
    mod.zero_grad(set_to_none=True)
    mod.training_step(data, 0).backward()
    torch.cuda.synchronize()
ka = prof.key_averages()
print(ka.table(sort_by="self_device_time_total", row_limit=45, max_name_column_width=60))
print(prof.key_averages(group_by_input_shape=True).table(sort_by="self_device_time_total",
                                                         row_limit=40, max_name_column_width=50,
                                                         max_shapes_column_width=70))
