"""fp64 companion of model_train_b2.npz: the oracle (bit-identical to the reference in fp32,
tests/golden/make_golden.py) re-run with fp64 arithmetic everywhere except the integer
pillar geometry (which stays fp32, as in the reference).

Deterministic-train mode (BN batch statistics at B=2) is ill-conditioned: the reference's
own fp32 result differs from this fp64 value by ~1e-3 on the segmentation logits and ~2 %
on some weight gradients (the cumsum-difference pooling noise, SURVEY.md §0 fact 4, is
amplified by batch-statistic BN).  Parity tests therefore measure both the product and the
reference against this fp64 value.   Run: python tests/golden/make_fp64.py [b8|c4|c4b4]
(b8: the same for the B=8 bench batch, model_train_b8.npz; c4: model_train_c4.npz.)
"""
import os
import sys

import numpy as np
import torch

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
sys.path[:0] = [REPO, os.path.join(REPO, "tests"), os.path.join(REPO, "e2e-parking-carla_amd")]

from oracle import parking_ref as O  # noqa: E402
from e2ep_amd import synthetic  # noqa: E402
from weights import make_grad_probe_keys, make_state  # noqa: E402


def oracle_model(dtype, cfg=O.Cfg):
    torch.manual_seed(0)
    m = O.ParkingModelRef(cfg, dropout=False)
    m.load_state_dict(make_state(m.state_dict(), 1234))
    keep = {k: v.detach().clone() for k, v in m.bev_model.named_parameters(recurse=False)}
    m = m.to(dtype)
    for k, v in keep.items():  # geometry constants stay fp32 (integer pillar index)
        getattr(m.bev_model, k).data = v
    return m


def sample(t):
    """make_golden.sample: every k-th element, k = max(1, numel // 16384)."""
    flat = t.detach().reshape(-1)
    return flat[::max(1, flat.numel() // 16384)].clone()


def main_b8():
    """fp64 companion of model_train_b8.npz (same batch / noise seeds, same sampling)."""
    import json
    torch.set_num_threads(8)
    m = oracle_model(torch.float64).train()
    data = synthetic.synthetic_batch(8, seed=11)
    noise = synthetic.target_noise(8, seed=11)
    d = {k: (v.double() if v.is_floating_point() and k not in ("intrinsics", "extrinsics") else v)
         for k, v in data.items()}
    losses, (pc, ps, pd) = O.train_losses(m, d, noise)
    losses["train_loss"].backward()
    with open(os.path.join(HERE, "meta.json")) as f:
        gkeys = json.load(f)["model_train_b8"]["grad_keys"]
    params = dict(m.named_parameters())
    fx = {"loss_control": np.float64(losses["control_loss"].item()),
          "loss_seg": np.float64(losses["segmentation_loss"].item()),
          "loss_depth": np.float64(losses["depth_loss"].item()),
          "pred_control": pc.detach().numpy(),
          "seg_sample": sample(ps).numpy(), "seg_norm": np.float64(ps.detach().norm()),
          "depth_sample": sample(pd).numpy(), "depth_norm": np.float64(pd.detach().norm()),
          "gnorm_all": np.array([float(params[k].grad.norm()) for k in gkeys])}
    for k in make_grad_probe_keys(params.keys()):
        fx["gsample::" + k] = sample(params[k].grad).numpy()
    np.savez_compressed(os.path.join(HERE, "model_train_b8_fp64.npz"), **fx)
    print("wrote model_train_b8_fp64.npz")
    # eval-mode gradients (model_evalgrad_b8.npz)
    m = oracle_model(torch.float64).eval()
    losses, _ = O.train_losses(m, d, noise)
    losses["train_loss"].backward()
    with open(os.path.join(HERE, "meta.json")) as f:
        gkeys = json.load(f)["model_evalgrad_b8"]["grad_keys"]
    params = dict(m.named_parameters())
    fx = {"loss_control": np.float64(losses["control_loss"].item()),
          "loss_seg": np.float64(losses["segmentation_loss"].item()),
          "loss_depth": np.float64(losses["depth_loss"].item()),
          "gnorm_all": np.array([float(params[k].grad.norm()) for k in gkeys])}
    for k in make_grad_probe_keys(params.keys()):
        fx["gsample::" + k] = sample(params[k].grad).numpy()
    np.savez_compressed(os.path.join(HERE, "model_evalgrad_b8_fp64.npz"), **fx)
    print("wrote model_evalgrad_b8_fp64.npz")


def main():
    torch.set_num_threads(8)
    m = oracle_model(torch.float64).train()
    data = synthetic.synthetic_batch(2, seed=5)
    noise = synthetic.target_noise(2, seed=5)
    d = {k: (v.double() if v.is_floating_point() and k not in ("intrinsics", "extrinsics") else v)
         for k, v in data.items()}
    losses, (pc, ps, pd) = O.train_losses(m, d, noise)
    losses["train_loss"].backward()
    fx = {"loss_control": np.float64(losses["control_loss"].item()),
          "loss_seg": np.float64(losses["segmentation_loss"].item()),
          "loss_depth": np.float64(losses["depth_loss"].item()),
          "pred_control": pc.detach().numpy(), "seg_norm": np.float64(ps.detach().norm()),
          "seg_slice": ps.detach()[:, :, 90:110, 90:110].numpy(),
          "depth_norm": np.float64(pd.detach().norm()), "depth_slice": pd.detach()[:, :, 10:14].numpy()}
    params = dict(m.named_parameters())
    for k in make_grad_probe_keys(params.keys()):
        g = params[k].grad.reshape(-1)
        fx["gnorm::" + k] = np.float64(g.norm())
        fx["gslice::" + k] = g[:4096].numpy()
    np.savez_compressed(os.path.join(HERE, "model_train_b2_fp64.npz"), **fx)
    print("wrote model_train_b2_fp64.npz")


def main_c4():
    """fp64 companion of model_train_c4.npz (C4: 6 cameras at 512x512, B=1)."""
    torch.set_num_threads(8)

    class CfgC4(O.Cfg):
        final_dim = [512, 512]

    import json
    with open(os.path.join(HERE, "meta.json")) as f:
        meta = json.load(f)
    data = synthetic.synthetic_batch(1, seed=13, hires=True)
    noise = synthetic.target_noise(1, seed=13)
    d = {k: (v.double() if v.is_floating_point() and k not in ("intrinsics", "extrinsics") else v)
         for k, v in data.items()}
    for mode, name in (("train", "model_train_c4"), ("eval", "model_evalgrad_c4")):
        m = oracle_model(torch.float64, CfgC4)
        m.train(mode == "train")
        losses, (pc, ps, pd) = O.train_losses(m, d, noise)
        losses["train_loss"].backward()
        params = dict(m.named_parameters())
        fx = {"loss_control": np.float64(losses["control_loss"].item()),
              "loss_seg": np.float64(losses["segmentation_loss"].item()),
              "loss_depth": np.float64(losses["depth_loss"].item()),
              "gnorm_all": np.array([float(params[k].grad.norm()) for k in meta[name]["grad_keys"]])}
        if mode == "train":
            fx.update(pred_control=pc.detach().numpy(),
                      seg_slice=ps.detach()[:, :, 90:110, 90:110].numpy(),
                      depth_slice=pd.detach()[:, :, 10:14].numpy())
        np.savez_compressed(os.path.join(HERE, name + "_fp64.npz"), **fx)
        print("wrote", name + "_fp64.npz")


def main_c4b4():
    """fp64 companion of model_train_c4b4.npz (C4 at the benched B=4, deterministic train)."""
    import json
    torch.set_num_threads(8)

    class CfgC4(O.Cfg):
        final_dim = [512, 512]

    with open(os.path.join(HERE, "meta.json")) as f:
        info = json.load(f)["model_train_c4b4"]
    data = synthetic.synthetic_batch(4, seed=17, hires=True)
    noise = synthetic.target_noise(4, seed=17)
    d = {k: (v.double() if v.is_floating_point() and k not in ("intrinsics", "extrinsics") else v)
         for k, v in data.items()}
    m = oracle_model(torch.float64, CfgC4).train()
    # 24 images at 512^2 in fp64 keep > 60 GB of activations for the backward: recompute each
    # EfficientNet block in the backward instead (same arithmetic; no dropout / drop-connect in
    # this protocol, so the recomputed forward is the forward)
    from torch.utils.checkpoint import checkpoint
    for blk in m.bev_model.cam_encoder.backbone._blocks:
        blk.forward = (lambda f: lambda x, drop_connect_rate=None: checkpoint(
            f, x, drop_connect_rate, use_reentrant=False))(blk.forward)
    losses, (pc, ps, pd) = O.train_losses(m, d, noise)
    losses["train_loss"].backward()
    params = dict(m.named_parameters())
    fx = {"loss_control": np.float64(losses["control_loss"].item()),
          "loss_seg": np.float64(losses["segmentation_loss"].item()),
          "loss_depth": np.float64(losses["depth_loss"].item()),
          "pred_control": pc.detach().numpy(),
          "seg_sample": sample(ps).numpy(), "depth_sample": sample(pd).numpy(),
          "gnorm_all": np.array([float(params[k].grad.norm()) for k in info["grad_keys"]])}
    for k in info["probe"]:
        fx["gsample::" + k] = sample(params[k].grad).numpy()
    np.savez_compressed(os.path.join(HERE, "model_train_c4b4_fp64.npz"), **fx)
    print("wrote model_train_c4b4_fp64.npz")


if __name__ == "__main__":
    if len(sys.argv) > 1 and sys.argv[1] == "b8":
        main_b8()
    elif len(sys.argv) > 1 and sys.argv[1] == "c4":
        main_c4()
    elif len(sys.argv) > 1 and sys.argv[1] == "c4b4":
        main_c4b4()
    else:
        main()
