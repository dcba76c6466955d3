import os, sys
ROOT = "/root/repo" if os.path.exists("/root/repo") else os.environ["GRAFT_REPO_ROOT"]
sys.path[:0] = [os.path.join(ROOT, "e2e-parking-carla_amd"), ROOT]
import torch
from torch.profiler import ProfilerActivity, profile
from model.control_predict import ControlPredict
from model.feature_fusion import FeatureFusion
from tool.config import default_cfg
cfg = default_cfg(); dev = torch.device("cuda")
ff = FeatureFusion(cfg).to(dev).train(); cp = ControlPredict(cfg).to(dev).train()
B = 8
bev = torch.randn(B, 256, 256, device=dev, requires_grad=True)
ego = torch.randn(B, 1, 3, device=dev)
gt = torch.randint(0, 200, (B, 15), device=dev)
def step():
    fused = ff(bev, ego); out = cp(fused, gt)
    (out.square().mean() + fused.square().mean()).backward()
for _ in range(3): step()
torch.cuda.synchronize()
with profile(activities=[ProfilerActivity.CPU, ProfilerActivity.CUDA]) as prof:
    step(); torch.cuda.synchronize()
print(prof.key_averages().table(sort_by="cuda_time_total", row_limit=60, max_name_column_width=55))
