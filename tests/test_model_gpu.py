"""Full ParkingModel on MI355X vs golden vectors from the reference (closed-form weights).

Tolerances (BASELINE north_star): rel-L2 <= 1e-4 per output; the integer
outputs (predicted control tokens, target plane) must be identical."""
import numpy as np
import pytest
import torch

from helpers import golden, rel_l2

pytestmark = pytest.mark.gpu
DEV = "cuda"
TOL = 1e-4


def _model(deterministic):
    from model.parking_model import ParkingModel
    from tool.config import default_cfg
    from weights import make_state
    m = ParkingModel(default_cfg(deterministic=deterministic))
    m.load_state_dict(make_state(m.state_dict(), 1234))
    return m.to(DEV)


def test_eval_forward_and_predict_match_reference():
    from e2ep_amd import synthetic
    g = golden("model_eval_b1.npz")
    m = _model(True).eval()
    data = synthetic.synthetic_batch(1, seed=3)
    noise = synthetic.target_noise(1, seed=3).to(DEV)
    with torch.no_grad():
        pc, ps, pd = m(data, noise)
        tok, _, _, tgt = m.predict({**data, "gt_control": data["gt_control"][:, :1]}, noise)
    assert rel_l2(pc, g["pred_control"]) < TOL
    assert rel_l2(ps, g["pred_segmentation"]) < TOL
    assert rel_l2(pd, g["pred_depth"]) < TOL
    assert np.array_equal(tok.cpu().numpy(), g["predict_tokens"])
    assert np.array_equal(tgt.cpu().numpy(), g["bev_target"])


def test_deterministic_train_step_matches_reference():
    from e2ep_amd import synthetic
    from trainer.pl_trainer import ParkingTrainingModule
    from tool.config import default_cfg
    from weights import make_grad_probe_keys, make_state
    g = golden("model_train_b2.npz")
    mod = ParkingTrainingModule(default_cfg(deterministic=True))
    mod.parking_model.load_state_dict(make_state(mod.parking_model.state_dict(), 1234))
    mod = mod.to(DEV).train()
    data = synthetic.synthetic_batch(2, seed=5)
    noise = synthetic.target_noise(2, seed=5).to(DEV)
    losses, (pc, ps, pd) = mod.compute_losses(data, noise)
    losses["train_loss"].backward()
    for k, gk in (("control_loss", "loss_control"), ("segmentation_loss", "loss_seg"), ("depth_loss", "loss_depth")):
        assert abs(float(losses[k]) / float(g[gk]) - 1) < TOL, k
    assert rel_l2(pc, g["pred_control"]) < TOL
    assert abs(float(ps.double().norm()) / float(g["seg_norm"]) - 1) < TOL
    assert rel_l2(ps[:, :, 90:110, 90:110], g["seg_slice"]) < TOL
    assert rel_l2(pd[:, :, 10:14], g["depth_slice"]) < TOL
    params = dict(mod.parking_model.named_parameters())
    for k in make_grad_probe_keys(params.keys()):
        gk = params[k].grad.reshape(-1)
        assert abs(float(gk.double().norm()) / float(g["gnorm::" + k]) - 1) < 1e-3, k
        assert rel_l2(gk[:4096], g["gslice::" + k]) < 1e-3, k
