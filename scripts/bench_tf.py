"""Microbenchmark + kernel census of the transformer stacks (FeatureFusion encoder, 4 layers,
B x 256 x 258; ControlPredict decoder, 4 layers, B x 14 x 258, memory 256) fwd+bwd, train mode.
    python scripts/bench_tf.py [--batch 8] [--iters 20]"""
import argparse
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "e2e-parking-carla_amd"), ROOT]
import torch  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=8)
    ap.add_argument("--iters", type=int, default=20)
    a = ap.parse_args()
    from model.control_predict import ControlPredict
    from model.feature_fusion import FeatureFusion
    from tool.config import default_cfg
    cfg = default_cfg()
    dev = torch.device("cuda")
    ff = FeatureFusion(cfg).to(dev).train()
    cp = ControlPredict(cfg).to(dev).train()
    B = a.batch
    bev = torch.randn(B, 256, 256, device=dev, requires_grad=True)
    ego = torch.randn(B, 1, 3, device=dev)
    gt = torch.randint(0, 200, (B, 15), device=dev)

    def step():
        fused = ff(bev, ego)
        out = cp(fused, gt)
        (out.square().mean() + fused.square().mean()).backward()

    for _ in range(3):
        step()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(a.iters):
        step()
    e.record()
    torch.cuda.synchronize()
    print(f"transformer fwd+bwd B={B}: {s.elapsed_time(e) / a.iters:.3f} ms/iter (eager)")


if __name__ == "__main__":
    main()
