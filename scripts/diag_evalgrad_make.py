"""Diagnostic fixtures: eval-mode gradient norms of the reference (fp32) and the oracle (fp64)
for a given rig / batch, per loss term (all / control / seg / depth), from the reference
itself (build container only): python scripts/diag_evalgrad_make.py c2|c4 B -> diag_tmp/.
The GPU side is scripts/diag_evalgrad_run.py (results: profiles/r02/session6/diag_*.json)."""
import os
import sys

import numpy as np
import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(REPO, "tests", "golden"), REPO, os.path.join(REPO, "e2e-parking-carla_amd"),
                os.path.join(REPO, "tests")]
import make_golden as MG  # noqa: E402
from oracle import parking_ref as O  # noqa: E402
from e2ep_amd import synthetic  # noqa: E402
from weights import make_state  # noqa: E402


def main():
    rig, B = sys.argv[1], int(sys.argv[2])
    hires = rig == "c4"
    MG.install_shims()
    torch.set_num_threads(8)
    import yaml
    from tool.config import get_cfg
    from model.parking_model import ParkingModel
    from loss.control_loss import ControlLoss
    from loss.seg_loss import SegmentationLoss
    from loss.depth_loss import DepthLoss
    with open(os.path.join(MG.REF, "config", "training.yaml")) as f:
        cfg = get_cfg(yaml.safe_load(f))
    cfg.device = torch.device("cpu")
    if hires:
        cfg.final_dim, cfg.image_crop = [512, 512], 512
    torch.manual_seed(0)
    ref = ParkingModel(cfg)
    state = make_state(ref.state_dict(), seed=1234)
    ref.load_state_dict(state)
    MG.deterministic(ref)
    ref.eval()
    data = synthetic.synthetic_batch(B, seed=13, hires=hires)
    noise = synthetic.target_noise(B, seed=13)
    with MG.FixedRand(noise):
        pc, ps, pd = ref(data)
    closs, dloss = ControlLoss(cfg), DepthLoss(cfg)
    sloss = SegmentationLoss(class_weights=torch.Tensor(cfg.seg_vehicle_weights))
    lc, ls, ld = closs(pc, data), sloss(ps.unsqueeze(1), data["segmentation"]), dloss(pd, data["depth"])
    parts = {"control": lc, "seg": ls, "depth": ld}
    out = {}
    keys = None
    for part in ("all",) + tuple(parts):
        ref.zero_grad(set_to_none=True)
        with MG.FixedRand(noise):
            pc, ps, pd = ref(data)
        lc, ls, ld = closs(pc, data), sloss(ps.unsqueeze(1), data["segmentation"]), dloss(pd, data["depth"])
        loss = {"all": lc + ls + ld, "control": lc, "seg": ls, "depth": ld}[part]
        loss.backward()
        g = dict(ref.named_parameters())
        if keys is None:
            keys = [k for k, v in g.items() if v.grad is not None]
        out["n32_" + part] = np.array([float(g[k].grad.double().norm()) if g[k].grad is not None else 0.0 for k in keys])

    class C(O.Cfg):
        final_dim = [512, 512] if hires else [256, 256]

    for part in ("all", "control", "seg", "depth"):
        torch.manual_seed(0)
        m = O.ParkingModelRef(C, dropout=False)
        m.load_state_dict(state)
        keep = {k: v.detach().clone() for k, v in m.bev_model.named_parameters(recurse=False)}
        m = m.double()
        for k, v in keep.items():
            getattr(m.bev_model, k).data = v
        m.eval()
        d = {k: (v.double() if v.is_floating_point() and k not in ("intrinsics", "extrinsics") else v)
             for k, v in data.items()}
        losses, _ = O.train_losses(m, d, noise)
        loss = {"all": losses["train_loss"], "control": losses["control_loss"],
                "seg": losses["segmentation_loss"], "depth": losses["depth_loss"]}[part]
        loss.backward()
        g = dict(m.named_parameters())
        out["n64_" + part] = np.array([float(g[k].grad.norm()) if g[k].grad is not None else 0.0 for k in keys])
    os.makedirs(os.path.join(REPO, "diag_tmp"), exist_ok=True)  # git-ignored, shipped to the box
    np.savez(os.path.join(REPO, "diag_tmp", f"evalgrad_{rig}_b{B}.npz"), keys=np.array(keys), **out)
    print("wrote", rig, B)


if __name__ == "__main__":
    main()
