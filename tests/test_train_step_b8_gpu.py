"""The benched kernel sequence, oracle-checked: the HIP-graph-captured TrainStep at the bench
configuration (B=8, 4 x 256^2, side-stream weight gradients on, exactly what bench.py
replays) against the reference's B=8 goldens, and the C3 (bf16 operand) train step against the
same goldens.

Reference: trainer/pl_trainer.py:55-83 (training_step: the three losses, their sum, backward)
on the make_golden.py b8 batch (synthetic_batch(8, seed=11), target noise seed 11, weights
make_state(1234), deterministic-train protocol: BN batch statistics, dropout / drop-connect 0).

Captured-step protocol.  TrainStep captures forward + losses + backward into g_bwd and the
Adam update into g_opt after `warmup` eager steps (which move the weights).  The test then
copies the initial weights back into the SAME parameter storage (the graph reads them by
address), replays g_bwd once and reads the gradients the replay wrote into the captured
.grad tensors — the gradients of the initial weights, comparable with the golden under the
rule tests/test_model_b8_gpu.py uses (per tensor: max(1e-4, 3 x the fp32 reference's own
error vs fp64)).

C3 comparator and bounds.  The reference has no bf16 mode (the whole model under
torch.autocast raises in model/bev_model.py:103), so make_golden.py b8bf16 runs the reference
the way a bf16 mixed-precision trainer runs the layers C3 puts on bf16 operands: its camera
encoder, BEV encoder and segmentation head (conv GEMMs) and its feature-fusion encoder and
control decoder (linear / attention projections; the product's C3 mode runs the transformer
linears on bf16 operands since round 3) under torch.autocast(bfloat16); lift-splat, the depth
softmax and the losses fp32; fp32 gradients (model_train_b8_bf16amp.npz).  Its error against
the fp64 oracle is the bf16 error budget:
  * the three losses: within max(1e-4, 3 x the AMP reference's error) of fp64;
  * probe-gradient samples: rel-L2 within 1.5 x the AMP reference's error;
  * gradient norms of all 530 parameters, as a set: median and max no larger than the AMP
    reference's (the product keeps bf16 only in the MFMA operands, fp32 in HBM, so it stays
    below AMP: round 3 measured median 0.020 vs 0.027, max 0.73 vs 4.0 against the
    conv-modules-only comparator; this comparator's own budget is median 0.032, max 4.1),
    and no larger than the product's own round-5 record with headroom (median 0.020, max
    1.0; measured 0.0160 / 0.722).
"""
import numpy as np
import pytest
import torch

from helpers import golden, meta, rel_l2
from test_model_b8_gpu import _check3, _norms3, _record, _scalar3, sample

pytestmark = pytest.mark.gpu
DEV = "cuda"


def _module():
    from trainer.pl_trainer import ParkingTrainingModule
    from tool.config import default_cfg
    from weights import make_state
    from e2ep_amd import synthetic
    mod = ParkingTrainingModule(default_cfg(deterministic=True))
    mod.parking_model.load_state_dict(make_state(mod.parking_model.state_dict(), 1234))
    mod = mod.to(DEV).train()
    for p in mod.parking_model.bev_encoder.layer4.parameters():  # as bench.py
        p.requires_grad_(False)
    noise = synthetic.target_noise(8, seed=11).to(DEV)
    mod.parking_model._noise = lambda b, device, n: noise  # the golden's target jitter
    return mod


def _batch(seed=11):
    from e2ep_amd import synthetic
    d = synthetic.synthetic_batch(8, seed=seed)
    # the rig stays on the host, as the data loader delivers it (memoised pillar plan)
    return {k: (v if k in ("intrinsics", "extrinsics") else v.to(DEV)) for k, v in d.items()}


def _captured_initial_grads(mod, warmup=2):
    """Capture the bench's TrainStep, restore the initial weights in place, replay the
    forward/backward graph once.  Returns (step, losses dict)."""
    from e2ep_amd import conv
    from e2ep_amd.train import TrainStep
    assert conv.wgrad_overlap(), "the bench replays the side-stream weight gradients"
    init = {k: v.detach().clone() for k, v in mod.parking_model.state_dict().items()}
    step = TrainStep(mod, _batch(), graph=True, warmup=warmup)
    with torch.no_grad():
        for k, v in mod.parking_model.state_dict().items():
            v.copy_(init[k])  # same storage: the captured graph reads these addresses
    step.g_bwd.replay()
    torch.cuda.synchronize()
    return step, {k: v.clone() for k, v in mod.logged.items()}


_PAIRS = (("control_loss", "loss_control"), ("segmentation_loss", "loss_seg"),
          ("depth_loss", "loss_depth"))


def test_captured_b8_step_gradients_match_reference():
    g32, g64 = golden("model_train_b8.npz"), golden("model_train_b8_fp64.npz")
    info = meta()["model_train_b8"]
    mod = _module()
    _, losses = _captured_initial_grads(mod)
    for k, gk in _PAIRS:
        _scalar3("captured_train_b8", gk, losses[k], g32[gk], g64[gk])
    params = dict(mod.parking_model.named_parameters())
    for k in info["probe"]:
        _check3("captured_train_b8", "grad " + k, sample(params[k].grad), g32["gsample::" + k],
                g64["gsample::" + k])
    _norms3("captured_train_b8", info["grad_keys"], params, g32["gnorm_all"], g64["gnorm_all"])


def test_captured_b8_step_matches_eager():
    """Graph replay at the bench shape (B=8 split-K / tile plans, forked weight-gradient
    branches) against the same steps run eagerly: two full steps (fwd, losses, bwd, Adam)."""
    from e2ep_amd.train import TrainStep
    m_e, m_g = _module(), _module()
    warm = 2
    s_e = TrainStep(m_e, _batch(), graph=False)
    s_g = TrainStep(m_g, _batch(), graph=True, warmup=warm)
    for _ in range(warm):
        s_e()
    le = [float(s_e()) for _ in range(2)]
    lg = [float(s_g()) for _ in range(2)]
    worst = 0.0
    for a, b in zip(le, lg):
        worst = max(worst, abs(a / b - 1))
    pe = dict(m_e.named_parameters())
    pworst = max(rel_l2(p.detach(), pe[k].detach()) for k, p in m_g.named_parameters())
    _record("captured_vs_eager_b8", "two_steps", loss_rel_max=worst, param_rel_l2_max=pworst)
    assert worst < 1e-6, (le, lg)
    assert lg[1] != lg[0]
    assert pworst < 1e-6


def test_bf16_b8_train_step_vs_reference():
    """C3: bf16 conv-GEMM operands (fwd, dgrad, wgrad), captured step, vs fp64 within the bf16
    AMP reference's own error (module docstring)."""
    from e2ep_amd import precision
    g32, g64 = golden("model_train_b8.npz"), golden("model_train_b8_fp64.npz")
    amp = golden("model_train_b8_bf16amp.npz")
    info = meta()["model_train_b8"]
    sec = "bf16_train_b8"
    with precision.use("bf16"):
        mod = _module()
        _, losses = _captured_initial_grads(mod)
    bad = []
    for k, gk in _PAIRS:
        e64 = abs(float(losses[k]) / float(g64[gk]) - 1)
        eamp = abs(float(amp[gk]) / float(g64[gk]) - 1)
        bound = max(1e-4, 3 * eamp)
        _record(sec, gk, vs_fp64=e64, amp_vs_fp64=eamp, bound=bound)
        if e64 > bound:
            bad.append((gk, e64, bound))
    params = dict(mod.parking_model.named_parameters())
    for k in info["probe"]:
        e64 = rel_l2(sample(params[k].grad), g64["gsample::" + k])
        eamp = rel_l2(amp["gsample::" + k], g64["gsample::" + k])
        _record(sec, "grad " + k, vs_fp64=e64, amp_vs_fp64=eamp,
                fp32_ref_vs_fp64=rel_l2(g32["gsample::" + k], g64["gsample::" + k]))
        if e64 > 1.5 * eamp:
            bad.append((k, e64, 1.5 * eamp))
    gk = info["grad_keys"]
    got = np.array([float(params[k].grad.double().norm()) for k in gk])
    n64 = g64["gnorm_all"]
    den = np.maximum(n64, 1e-3 * float(np.sqrt(np.mean(n64 ** 2))))
    e64 = np.abs(got - n64) / den
    eamp = np.abs(amp["gnorm_all"] - n64) / den
    _record(sec, "grad_norms(all %d)" % len(gk), vs_fp64_max=e64.max(),
            vs_fp64_median=np.median(e64), amp_vs_fp64_max=eamp.max(),
            amp_vs_fp64_median=np.median(eamp))
    for i in np.argsort(-e64)[:8]:
        _record(sec + "_worst", gk[i], vs_fp64=e64[i], amp_vs_fp64=eamp[i])
    if np.median(e64) > np.median(eamp):
        bad.append(("grad-norm median", np.median(e64), np.median(eamp)))
    if e64.max() > eamp.max():
        bad.append(("grad-norm max", e64.max(), eamp.max()))
    # second, tighter gate: the product's own measured margin.  The comparator
    # with the transformer under autocast widened the AMP budget (median 0.027 -> 0.032, max
    # 4.0 -> 4.1); the product measured median 0.0160 / max 0.722 (round 5,
    # profiles/r05/parity_bf16_b8.json), held here with 25 % / 40 % headroom.
    if np.median(e64) > 0.020:
        bad.append(("grad-norm median vs product record", np.median(e64), 0.020))
    if e64.max() > 1.0:
        bad.append(("grad-norm max vs product record", e64.max(), 1.0))
    assert not bad, bad


def test_captured_step_with_device_rig_equals_eager():
    """A rig that arrives as DEVICE tensors, in a capture-only process (warmup=0: the first
    step is the captured one): TrainStep plans the rig before the capture with the reference's
    fp32 host algebra (BevModel.prepare_capture), so the captured step trains on the same
    pillar table as the eager step and the two agree bit for bit after two steps (round 5
    planned inside the capture with the fp64 device algebra and only bounded the divergence).
    A batch with a different device rig is refused by the captured step."""
    from e2ep_amd import _lib
    from e2ep_amd.train import TrainStep
    batch = _batch()
    dev_batch = dict(batch, intrinsics=batch["intrinsics"].to(DEV),
                     extrinsics=batch["extrinsics"].to(DEV))
    m_e, m_g = _module(), _module()
    s_e = TrainStep(m_e, dict(dev_batch), graph=False)
    s_g = TrainStep(m_g, dict(dev_batch), graph=True, warmup=0)
    le = [float(s_e()) for _ in range(2)]
    lg = [float(s_g()) for _ in range(2)]
    torch.cuda.synchronize()
    pe = dict(m_e.named_parameters())
    worst = max(rel_l2(p.detach(), pe[k].detach()) for k, p in m_g.named_parameters())
    _record("device_rig_captured_vs_eager", "two_steps", loss1_rel=abs(le[0] / lg[0] - 1),
            loss2_rel=abs(le[1] / lg[1] - 1), param_rel_l2_max=worst)
    assert le == lg, (le, lg)
    assert all(torch.equal(p.detach(), pe[k].detach()) for k, p in m_g.named_parameters())
    moved = dict(dev_batch, extrinsics=dev_batch["extrinsics"].clone())
    moved["extrinsics"][0, 0, 0, 3] += 0.25
    with pytest.raises(_lib.E2EPError, match="different intrinsics/extrinsics"):
        s_g(moved)
    s_g(dict(dev_batch))  # the captured rig itself is accepted
