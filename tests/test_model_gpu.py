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


def _within_reference_noise(name, got, ref32, ref64, floor=TOL):
    """Product error vs the fp64 oracle must stay within the reference's own fp32 error (x2),
    or under the 1e-4 contract when the reference is better conditioned than that."""
    e_prod, e_ref = rel_l2(got, ref64), rel_l2(ref32, ref64)
    assert e_prod <= max(floor, 2.0 * e_ref), f"{name}: product {e_prod:.2e} vs reference {e_ref:.2e}"


def _scalar_rel(a, b):
    return abs(float(a) / float(b) - 1)


def test_deterministic_train_step_matches_reference():
    """Deterministic-train protocol at B=2.  BN batch statistics make this
    mode ill-conditioned: the reference's own fp32 result is ~1e-3 (seg) to ~2e-2 (some
    weight grads) away from the fp64 value (tests/golden/make_fp64.py), so each output is
    held to max(1e-4, 2 x the reference's own error) against fp64."""
    from e2ep_amd import synthetic
    from trainer.pl_trainer import ParkingTrainingModule
    from tool.config import default_cfg
    from weights import make_grad_probe_keys, make_state
    g32 = golden("model_train_b2.npz")
    g64 = golden("model_train_b2_fp64.npz")
    mod = ParkingTrainingModule(default_cfg(deterministic=True))
    mod.parking_model.load_state_dict(make_state(mod.parking_model.state_dict(), 1234))
    mod = mod.to(DEV).train()
    data = synthetic.synthetic_batch(2, seed=5)
    noise = synthetic.target_noise(2, seed=5).to(DEV)
    losses, (pc, ps, pd) = mod.compute_losses(data, noise)
    losses["train_loss"].backward()
    for k, gk in (("control_loss", "loss_control"), ("segmentation_loss", "loss_seg"), ("depth_loss", "loss_depth")):
        e_prod, e_ref = _scalar_rel(losses[k], g64[gk]), _scalar_rel(g32[gk], g64[gk])
        assert e_prod <= max(TOL, 2 * e_ref), (k, e_prod, e_ref)
    _within_reference_noise("pred_control", pc, g32["pred_control"], g64["pred_control"])
    _within_reference_noise("seg_slice", ps[:, :, 90:110, 90:110], g32["seg_slice"], g64["seg_slice"])
    _within_reference_noise("depth_slice", pd[:, :, 10:14], g32["depth_slice"], g64["depth_slice"])
    params = dict(mod.parking_model.named_parameters())
    for k in make_grad_probe_keys(params.keys()):
        gk = params[k].grad.reshape(-1)
        _within_reference_noise("grad " + k, gk[:4096], g32["gslice::" + k], g64["gslice::" + k])


def test_bn_counters_batched_like_reference():
    """num_batches_tracked after three training forwards (the first per-layer, later ones
    batched into one launch): 3 on every BN that runs, 0 on the never-run bev_encoder.layer4
    (reference model/bev_encoder.py:21,23-36); the drop-connect path (non-deterministic
    config) runs too."""
    from e2ep_amd import synthetic
    from model.parking_model import ParkingModel
    from tool.config import default_cfg
    m = ParkingModel(default_cfg()).to(DEV).train()
    data = synthetic.synthetic_batch(2, seed=1)
    for _ in range(3):
        with torch.no_grad():
            pc, ps, pd = m(data)
    assert torch.isfinite(pc).all() and torch.isfinite(ps).all() and torch.isfinite(pd).all()
    counts = {k: int(v) for k, v in m.state_dict().items() if k.endswith("num_batches_tracked")}
    assert len(counts) > 90
    for k, v in counts.items():
        assert v == (0 if k.startswith("bev_encoder.layer4.") else 3), k


@pytest.mark.parametrize("mode,tol", [("fp16", 5e-3), ("bf16", 3e-2)])
def test_low_precision_predict_tokens_match_reference(mode, tol):
    """C5 (fp16 closed-loop inference) and the C3 forward precision: ParkingModel.predict with
    the conv GEMMs on fp16 / bf16 operands (e2ep_amd.precision), captured into a HIP graph and
    replayed, gives the reference's control tokens and target plane exactly; the segmentation
    and depth outputs stay within the format's rounding of the fp32 reference (rel-L2 `tol`:
    fp16 keeps 11 mantissa bits, bf16 8)."""
    from e2ep_amd import graphs, precision, synthetic
    g = golden("model_eval_b1.npz")
    m = _model(True).eval()
    data = synthetic.synthetic_batch(1, seed=3)
    noise = synthetic.target_noise(1, seed=3).to(DEV)
    pdata = {k: (v if k in ("intrinsics", "extrinsics") else v.to(DEV)) for k, v in data.items()}
    pdata["gt_control"] = pdata["gt_control"][:, :1]

    def call():
        with torch.no_grad():
            return m.predict(pdata, noise)
    with precision.use(mode):
        call()
        s = torch.cuda.Stream()
        s.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(s):
            call()
        torch.cuda.current_stream().wait_stream(s)
        torch.cuda.synchronize()
        graph, out, _ = graphs.capture(call)
        graph.replay()
        torch.cuda.synchronize()
    tok, ps, pd, tgt = out
    assert np.array_equal(tok.cpu().numpy(), g["predict_tokens"])
    assert np.array_equal(tgt.cpu().numpy(), g["bev_target"])
    e_seg, e_dep = rel_l2(ps, g["pred_segmentation"]), rel_l2(pd, g["pred_depth"])
    print(f"{mode} predict: seg rel-L2 {e_seg:.2e}, depth rel-L2 {e_dep:.2e}")
    assert e_seg < tol and e_dep < tol


def test_eval_bn_batch_equals_per_layer_statistics():
    """nn_ops.EvalBnBatch: the second and later no_grad forwards compute the fused BN
    consumers' eval statistics in one e2ep_bn_eval_multi launch; outputs are bitwise those of
    the first forward (per-layer e2ep_bn_stats), also after the running statistics change and
    under a captured graph; with autograd on the batch stays inactive."""
    from e2ep_amd import graphs, nn_ops, synthetic
    m = _model(True).eval()
    data = synthetic.synthetic_batch(1, seed=5)
    data = {k: (v if k in ("intrinsics", "extrinsics") else v.to(DEV)) for k, v in data.items()}
    noise = synthetic.target_noise(1, seed=5).to(DEV)
    with torch.no_grad():
        first = [t.clone() for t in m(data, noise)]
        assert m._eval_bn.recorded is not None and len(m._eval_bn.recorded) >= 40
        second = m(data, noise)
        assert all(torch.equal(a, b) for a, b in zip(first, second))
        # new running statistics: the batch launch reads them at every forward
        bns = m._eval_bn.recorded
        for b in bns:
            b.running_var.mul_(1.5).add_(0.01)
        m._eval_bn.recorded = None  # record again: per-layer statistics of the new values
        ref = [t.clone() for t in m(data, noise)]
        g, out, _ = graphs.capture(lambda: m(data, noise))
        g.replay()
        torch.cuda.synchronize()
        assert all(torch.equal(a, b) for a, b in zip(ref, out))
        assert not all(torch.equal(a, b) for a, b in zip(ref, first))
    assert nn_ops._eval_bn_stats(bns[0]) is None  # autograd on: no shared views
