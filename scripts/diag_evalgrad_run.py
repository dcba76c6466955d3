"""GPU side of scripts/diag_evalgrad_make.py: product eval-mode gradient norms per loss part vs
the reference fp32 / oracle fp64 norms.  python scripts/diag_evalgrad_run.py c2|c4 B"""
import json
import os
import sys

import numpy as np
import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "e2e-parking-carla_amd"), os.path.join(REPO, "tests")]


def main():
    rig, B = sys.argv[1], int(sys.argv[2])
    hires = rig == "c4"
    from e2ep_amd import synthetic
    from trainer.pl_trainer import ParkingTrainingModule
    from tool.config import default_cfg
    from weights import make_state
    fx = np.load(os.path.join(REPO, "diag_tmp", f"evalgrad_{rig}_b{B}.npz"))
    keys = [str(k) for k in fx["keys"]]
    cfg = default_cfg(deterministic=True, **({"final_dim": [512, 512], "image_crop": 512} if hires else {}))
    mod = ParkingTrainingModule(cfg)
    mod.parking_model.load_state_dict(make_state(mod.parking_model.state_dict(), 1234))
    mod = mod.cuda().eval()
    data = synthetic.synthetic_batch(B, seed=13, hires=hires)
    noise = synthetic.target_noise(B, seed=13).cuda()
    res = {}
    for part, lk in (("all", "train_loss"), ("control", "control_loss"), ("seg", "segmentation_loss"),
                     ("depth", "depth_loss")):
        mod.zero_grad(set_to_none=True)
        losses, _ = mod.compute_losses(data, noise)
        losses[lk].backward()
        p = dict(mod.parking_model.named_parameters())
        got = np.array([float(p[k].grad.double().norm()) if p[k].grad is not None else 0.0 for k in keys])
        n32, n64 = fx["n32_" + part], fx["n64_" + part]
        den = np.maximum(n64, 1e-3 * float(np.sqrt(np.mean(n64 ** 2))) + 1e-30)
        e64, eref = np.abs(got - n64) / den, np.abs(n32 - n64) / den
        order = np.argsort(-e64)[:12]
        res[part] = {"prod_vs_fp64_median": float(np.median(e64)), "ref_vs_fp64_median": float(np.median(eref)),
                     "prod_max": float(e64.max()), "ref_max": float(eref.max()),
                     "worst": [(keys[i], float(e64[i]), float(eref[i])) for i in order]}
        print(rig, B, part, {k: v for k, v in res[part].items() if k != "worst"})
    os.makedirs(os.path.join(REPO, "gpurun_out", "diag"), exist_ok=True)
    with open(os.path.join(REPO, "gpurun_out", "diag", f"res_{rig}_b{B}.json"), "w") as f:
        json.dump(res, f, indent=1)


if __name__ == "__main__":
    main()
