"""Full ParkingModel at BASELINE configs[3] (C4: 6 cameras at 512x512, 200x200x0.1 m BEV grid)
vs the reference, on MI355X, at B=1 (the oracle's CPU budget).

Fixtures: tests/golden/make_golden.py c4 (the reference's own fp32 CPU outputs, written by
importing /root/reference; the oracle reproduces them exactly) and make_fp64.py c4 (the
oracle re-run in fp64).  C4 exercises shapes the 4-camera 256^2 tests do not: 64x64 camera
feature maps (3.4 M frustum points), 256^2 stem maps, 512^2 depth labels, 6-image BN
statistics.  Achieved errors go to the E2EP_PARITY_REPORT JSON (sections eval_c4,
evalgrad_c4, train_c4) and stdout.

Bounds.  Eval forward: <= 1e-4 vs the fp32 reference (the north-star contract); tokens and
target plane identical.  Losses and train-mode outputs: within max(1e-4, 3 x the reference's
own fp32 error) of the fp64 oracle.  Gradient norms (all 530 parameters, eval mode and
deterministic train): the per-tensor rule of the bench config (tests/test_model_b8_gpu.py
_norms3: each tensor within max(1e-4, 3 x the reference's own error on it, or its median
error if larger) of fp64).

History: round 2 held C4's gradients only as a set, because the product was further from
fp64 than the reference there.  The cause was the pillar index: the device rig algebra (fp64
Gauss-Jordan) flipped 6 of the 1.18 M frustum points to a neighbouring cell against the
reference's fp32 LAPACK combine, and the fp64 oracle keeps the reference's fp32 geometry, so
those points moved BEV features the train-mode BN statistics then spread everywhere.  Host
rigs now go through the reference's own fp32 CPU algebra (bit-exact pillar table,
tests/test_lss_gpu.py::test_host_rig_pillar_index_bit_exact_end_to_end) and the product is
10-400 x closer to fp64 than the reference on every C4 output (profiles/r03/parity_c4.json)."""
import numpy as np
import pytest
import torch

from helpers import golden, meta, rel_l2
from test_model_b8_gpu import BOUND_FACTOR, TOL, _check3, _norms3, _record

pytestmark = pytest.mark.gpu
DEV = "cuda"


class _Checks:
    """Run every check, record every number, then fail with the list of violated bounds."""

    def __init__(self):
        self.failed = []

    def __call__(self, fn, *a):
        try:
            fn(*a)
        except AssertionError as e:
            self.failed.append(str(e)[:300])

    def done(self):
        assert not self.failed, self.failed


def _scalar(section, name, got, ref32, ref64):
    r = lambda a, b: abs(float(a) / float(b) - 1)  # noqa: E731
    e32, e64, eref = r(got, ref32), r(got, ref64), r(ref32, ref64)
    _record(section, name, vs_ref=e32, vs_fp64=e64, ref_vs_fp64=eref)
    assert e64 <= max(TOL, BOUND_FACTOR * eref), (section, name, e64, eref)


def _cfg():
    from tool.config import default_cfg
    return default_cfg(deterministic=True, final_dim=[512, 512], image_crop=512)


def _model():
    from model.parking_model import ParkingModel
    from weights import make_state
    m = ParkingModel(_cfg())
    m.load_state_dict(make_state(m.state_dict(), 1234))
    return m.to(DEV)


def _data():
    from e2ep_amd import synthetic
    return synthetic.synthetic_batch(1, seed=13, hires=True), synthetic.target_noise(1, seed=13).to(DEV)


def test_c4_eval_forward_and_predict_match_reference():
    g = golden("model_eval_c4.npz")
    m = _model().eval()
    data, noise = _data()
    with torch.no_grad():
        pc, ps, pd = m(data, noise)
        tok, _, _, tgt = m.predict({**data, "gt_control": data["gt_control"][:, :1]}, noise)
    errs = {"pred_control": rel_l2(pc, g["pred_control"]),
            "pred_segmentation": rel_l2(ps, g["pred_segmentation"]),
            "pred_depth": rel_l2(pd, g["pred_depth"])}
    for k, v in errs.items():
        _record("eval_c4", k, vs_ref=v)
    assert max(errs.values()) < TOL, errs
    assert np.array_equal(tok.cpu().numpy(), g["predict_tokens"])
    assert np.array_equal(tgt.cpu().numpy(), g["bev_target"])


def test_c4_eval_mode_gradients_match_reference():
    from trainer.pl_trainer import ParkingTrainingModule
    from weights import make_state
    g32, g64 = golden("model_evalgrad_c4.npz"), golden("model_evalgrad_c4_fp64.npz")
    mod = ParkingTrainingModule(_cfg())
    mod.parking_model.load_state_dict(make_state(mod.parking_model.state_dict(), 1234))
    mod = mod.to(DEV).eval()
    data, noise = _data()
    losses, _ = mod.compute_losses(data, noise)
    losses["train_loss"].backward()
    chk = _Checks()
    for k, gk in (("control_loss", "loss_control"), ("segmentation_loss", "loss_seg"),
                  ("depth_loss", "loss_depth")):
        chk(_scalar, "evalgrad_c4", gk, losses[k].detach(), g32[gk], g64[gk])
    chk(_norms3, "evalgrad_c4", meta()["model_evalgrad_c4"]["grad_keys"],
        dict(mod.parking_model.named_parameters()), g32["gnorm_all"], g64["gnorm_all"])
    chk.done()


def test_c4_deterministic_train_step_matches_reference():
    from trainer.pl_trainer import ParkingTrainingModule
    from weights import make_state
    g32, g64 = golden("model_train_c4.npz"), golden("model_train_c4_fp64.npz")
    mod = ParkingTrainingModule(_cfg())
    mod.parking_model.load_state_dict(make_state(mod.parking_model.state_dict(), 1234))
    mod = mod.to(DEV).train()
    data, noise = _data()
    losses, (pc, ps, pd) = mod.compute_losses(data, noise)
    losses["train_loss"].backward()
    chk = _Checks()
    for k, gk in (("control_loss", "loss_control"), ("segmentation_loss", "loss_seg"),
                  ("depth_loss", "loss_depth")):
        chk(_scalar, "train_c4", gk, losses[k].detach(), g32[gk], g64[gk])
    chk(_check3, "train_c4", "pred_control", pc, g32["pred_control"], g64["pred_control"])
    chk(_check3, "train_c4", "seg_slice", ps[:, :, 90:110, 90:110], g32["seg_slice"], g64["seg_slice"])
    chk(_check3, "train_c4", "depth_slice", pd[:, :, 10:14], g32["depth_slice"], g64["depth_slice"])
    chk(_norms3, "train_c4", meta()["model_train_c4"]["grad_keys"],
        dict(mod.parking_model.named_parameters()), g32["gnorm_all"], g64["gnorm_all"])
    chk.done()
