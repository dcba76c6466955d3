"""Full ParkingModel at BASELINE configs[3] (C4: 6 cameras at 512x512, 200x200x0.1 m BEV grid)
vs the reference, on MI355X: eager at B=1, and the benched step itself — the HIP-graph-captured
TrainStep at B=4 — against the reference's B=4 deterministic-train step and against eager.

Fixtures: tests/golden/make_golden.py c4 / c4b4 (the reference's own fp32 CPU outputs,
written by importing /root/reference; the oracle reproduces them exactly) and make_fp64.py
c4 / c4b4 (the oracle re-run in fp64; at B=4 with the EfficientNet blocks recomputed in the
backward to fit the container's memory).  C4 exercises shapes the 4-camera 256^2 tests do not: 64x64 camera
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


# ---- the benched C4 step: B=4, HIP-graph captured (bench.py secondary_c4) --------------------

def _train_module_b4():
    from trainer.pl_trainer import ParkingTrainingModule
    from weights import make_state
    from e2ep_amd import synthetic
    mod = ParkingTrainingModule(_cfg())
    mod.parking_model.load_state_dict(make_state(mod.parking_model.state_dict(), 1234))
    mod = mod.to(DEV).train()
    for p in mod.parking_model.bev_encoder.layer4.parameters():  # as bench.py
        p.requires_grad_(False)
    noise = synthetic.target_noise(4, seed=17).to(DEV)
    mod.parking_model._noise = lambda b, device, n: noise  # the golden's target jitter
    return mod


def _batch_b4():
    from e2ep_amd import synthetic
    d = synthetic.synthetic_batch(4, seed=17, hires=True)
    # the rig stays on the host, as the data loader delivers it (memoised pillar plan)
    return {k: (v if k in ("intrinsics", "extrinsics") else v.to(DEV)) for k, v in d.items()}


def test_c4_captured_b4_step_gradients_match_reference():
    """The captured B=4 C4 TrainStep (the C4 bench line's kernel sequence: B=4 split-K / tile
    plans, forked weight-gradient branches, BN statistics over 24 camera images) against the
    reference's deterministic-train step on the same batch (make_golden.py c4b4): losses,
    control logits, probe-gradient samples and all parameters' gradient norms, each within
    max(1e-4, 3 x the fp32 reference's own error vs fp64) of the fp64 oracle.  The initial
    weights are restored in place after capture and the forward/backward graph replayed once
    (tests/test_train_step_b8_gpu.py protocol)."""
    from e2ep_amd import conv
    from e2ep_amd.train import TrainStep
    from test_model_b8_gpu import _scalar3, sample
    g32, g64 = golden("model_train_c4b4.npz"), golden("model_train_c4b4_fp64.npz")
    info = meta()["model_train_c4b4"]
    assert conv.wgrad_overlap(), "the bench replays the side-stream weight gradients"
    mod = _train_module_b4()
    init = {k: v.detach().clone() for k, v in mod.parking_model.state_dict().items()}
    step = TrainStep(mod, _batch_b4(), graph=True, warmup=2)
    with torch.no_grad():
        for k, v in mod.parking_model.state_dict().items():
            v.copy_(init[k])  # same storage: the captured graph reads these addresses
    step.g_bwd.replay()
    torch.cuda.synchronize()
    losses = {k: v.clone() for k, v in mod.logged.items()}
    sec = "captured_train_c4b4"
    chk = _Checks()
    for k, gk in (("control_loss", "loss_control"), ("segmentation_loss", "loss_seg"),
                  ("depth_loss", "loss_depth")):
        chk(_scalar3, sec, gk, losses[k], g32[gk], g64[gk])
    params = dict(mod.parking_model.named_parameters())
    for k in info["probe"]:
        chk(_check3, sec, "grad " + k, sample(params[k].grad), g32["gsample::" + k],
            g64["gsample::" + k])
    chk(_norms3, sec, info["grad_keys"], params, g32["gnorm_all"], g64["gnorm_all"])
    chk.done()


def test_c4_captured_b4_step_matches_eager():
    """Graph replay of the benched C4 step (B=4) against the same steps run eagerly: two full
    steps (forward, losses, backward, Adam) after two warm-up steps."""
    from e2ep_amd.train import TrainStep
    m_e, m_g = _train_module_b4(), _train_module_b4()
    warm = 2
    s_e = TrainStep(m_e, _batch_b4(), graph=False)
    s_g = TrainStep(m_g, _batch_b4(), graph=True, warmup=warm)
    for _ in range(warm):
        s_e()
    le = [float(s_e()) for _ in range(2)]
    lg = [float(s_g()) for _ in range(2)]
    worst = max(abs(a / b - 1) for a, b in zip(le, lg))
    pe = dict(m_e.named_parameters())
    pworst = max(rel_l2(p.detach(), pe[k].detach()) for k, p in m_g.named_parameters())
    _record("captured_vs_eager_c4b4", "two_steps", loss_rel_max=worst, param_rel_l2_max=pworst)
    assert worst < 1e-6, (le, lg)
    assert lg[1] != lg[0]
    assert pworst < 1e-6
