"""Generate the golden vectors under tests/golden/ FROM THE REFERENCE ITSELF.

Run in the build container only (needs /root/reference):  python tests/golden/make_golden.py
(`python tests/golden/make_golden.py b8` regenerates only the B=8 fixtures, `... c4` adds the
C4 6-camera 512x512 fixtures, `... c4b4` the C4 deterministic-train step at the benched B=4,
`... b8bf16` the C3 bf16-autocast comparator.)

The reference has no tests or fixtures of its own, so every golden vector is
produced here by importing the reference's Python modules unmodified, with:
  * stubs for init-only / dead-code imports: timm.models.layers (trunc_normal_, DropPath),
    pyquaternion (dead code in tool/geometry.py:62-282);
  * the third-party trunks efficientnet_pytorch / torchvision.models.resnet, which are not
    installed, provided by the oracle's restatement (oracle/trunks.py) — so backbone parity
    against the real packages is UNPINNED;
  * runtime shims for torch-1.13-era code on a CPU-only box: np.int, Tensor.cuda -> identity,
    Tensor.to('cuda') -> cpu.
No reference source is copied; only inputs/outputs are written.  The script also asserts
that the oracle restatement (oracle/parking_ref.py) reproduces the reference on the same
inputs before it writes anything.
"""
import hashlib
import json
import os
import sys
import types

import numpy as np
import torch

REPO = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
REF = "/root/reference"
OUT = os.path.join(REPO, "tests", "golden")
sys.path.insert(0, REPO)
sys.path.insert(0, os.path.join(REPO, "e2e-parking-carla_amd"))
sys.path.insert(0, os.path.join(REPO, "tests"))

from oracle import trunks, parking_ref as O  # noqa: E402
from e2ep_amd import synthetic  # noqa: E402
from weights import make_state, make_grad_probe_keys  # noqa: E402


def install_shims():
    np.int = int
    timm = types.ModuleType("timm")
    tm = types.ModuleType("timm.models")
    tl = types.ModuleType("timm.models.layers")
    tl.trunc_normal_ = torch.nn.init.trunc_normal_
    tl.DropPath = lambda *a, **k: torch.nn.Identity()
    timm.models, tm.layers = tm, tl
    sys.modules.update({"timm": timm, "timm.models": tm, "timm.models.layers": tl})
    pq = types.ModuleType("pyquaternion")
    pq.Quaternion = object
    sys.modules["pyquaternion"] = pq
    eff = types.ModuleType("efficientnet_pytorch")
    eff.EfficientNet = trunks.EfficientNet
    sys.modules["efficientnet_pytorch"] = eff
    tv = types.ModuleType("torchvision")
    tvm = types.ModuleType("torchvision.models")
    tvr = types.ModuleType("torchvision.models.resnet")
    tvr.resnet18 = trunks.resnet18
    tv.models, tvm.resnet = tvm, tvr
    sys.modules.update({"torchvision": tv, "torchvision.models": tvm, "torchvision.models.resnet": tvr})
    torch.Tensor.cuda = lambda self, *a, **k: self
    orig_to = torch.Tensor.to

    def to(self, *a, **k):
        a = tuple("cpu" if (isinstance(x, str) and x.startswith("cuda")) else x for x in a)
        if isinstance(k.get("device"), str) and k["device"].startswith("cuda"):
            k["device"] = "cpu"
        return orig_to(self, *a, **k)

    torch.Tensor.to = to
    # the product tree mirrors the reference's package names (model, tool, loss, ...) as
    # regular packages, which would shadow the reference's namespace packages: take it off
    # the path (e2ep_amd.synthetic is already imported) so `model.*` is the reference's
    prod = os.path.join(REPO, "e2e-parking-carla_amd")
    sys.path[:] = [p for p in sys.path if os.path.abspath(p or ".") != prod]
    for name in list(sys.modules):
        if name.split(".")[0] in ("model", "tool", "loss", "trainer", "dataset"):
            del sys.modules[name]
    sys.path.insert(0, REF)


def deterministic(model):
    """SURVEY.md §8c deterministic-train protocol applied to a reference model instance."""
    for m in model.modules():
        if isinstance(m, torch.nn.Dropout):
            m.p = 0.0
        if isinstance(m, torch.nn.MultiheadAttention):
            m.dropout = 0.0
    gp = model.bev_model.cam_encoder.backbone._global_params
    model.bev_model.cam_encoder.backbone._global_params = gp._replace(drop_connect_rate=0.0)
    return model


class FixedRand:
    def __init__(self, noise):
        self.noise, self.orig = noise, torch.rand_like

    def __enter__(self):
        torch.rand_like = lambda t, dtype=None, **k: self.noise.to(dtype or torch.float).clone()

    def __exit__(self, *a):
        torch.rand_like = self.orig


def rel(a, b):
    a, b = a.double(), b.double()
    return float((a - b).norm() / max(b.norm(), 1e-30))


SAMPLE = 16384


def sample(t):
    """A strided subsample of a large output (every k-th element of the flattened tensor,
    k = max(1, numel // SAMPLE)); tests/test_model_b8_gpu.py recomputes the same indices."""
    flat = t.detach().reshape(-1)
    return flat[::max(1, flat.numel() // SAMPLE)].clone()


def b8_fixtures(ref, orc, state, cfg, closs, sloss, dloss, meta):
    """C2 bench workload (B=8, 4 x 256^2): eval forward + predict, and one deterministic-train
    forward/backward with the three losses.  Full control logits; strided samples + norms of
    the segmentation / depth outputs; every parameter's gradient norm and strided samples of
    the probe tensors' gradients."""
    B = 8
    data = synthetic.synthetic_batch(B, seed=11)
    noise = synthetic.target_noise(B, seed=11)
    ref.load_state_dict(state)
    orc.load_state_dict(state)
    ref.eval(), orc.eval()
    with torch.no_grad(), FixedRand(noise):
        pc, ps, pd = ref(data)
        tok, _, _, tgt = ref.predict({**data, "gt_control": data["gt_control"][:, :1]})
    with torch.no_grad():
        qc, qs, qd = orc(data, noise)
    errs = {"control": rel(qc, pc), "seg": rel(qs, ps), "depth": rel(qd, pd)}
    print("oracle vs reference, eval B=8:", errs)
    assert max(errs.values()) < 1e-6
    # validation_step arithmetic (trainer/pl_trainer.py:85-114) on the eval-mode outputs:
    # the reference's ControlValLoss / SegmentationLoss / DepthLoss modules
    from loss.control_loss import ControlValLoss
    with torch.no_grad():
        acc_steer, reverse = ControlValLoss(cfg)(pc, data)
        seg_v = sloss(ps.unsqueeze(1), data["segmentation"])
        dep_v = dloss(pd, data["depth"])
    val = {"acc_steer_val_loss": acc_steer, "reverse_val_loss": reverse,
           "segmentation_val_loss": seg_v, "depth_val_loss": dep_v}
    val["val_loss"] = sum(val.values())
    np.savez_compressed(os.path.join(OUT, "validation_b8.npz"),
                        **{k: np.float64(v) for k, v in val.items()})
    meta["validation_b8"] = {"batch_seed": 11, "noise_seed": 11, "mode": "eval"}
    np.savez_compressed(os.path.join(OUT, "model_eval_b8.npz"), pred_control=pc.numpy(),
                        seg_sample=sample(ps).numpy(), seg_norm=np.float64(ps.double().norm()),
                        depth_sample=sample(pd).numpy(), depth_norm=np.float64(pd.double().norm()),
                        predict_tokens=tok.numpy(), bev_target_sum=tgt.sum((1, 2, 3)).numpy())
    meta["model_eval_b8"] = {"batch_seed": 11, "noise_seed": 11, "oracle_rel_err": errs,
                             "sample": SAMPLE}

    deterministic(ref)
    probe = make_grad_probe_keys(state.keys())
    # (3c') gradients in eval mode (BN on running statistics): the whole backward without the
    # batch-statistic BN conditioning of train mode -- a well-conditioned gradient check
    ref.load_state_dict(state)
    ref.eval()
    with FixedRand(noise):
        pc, ps, pd = ref(data)
    lc, ls, ld = closs(pc, data), sloss(ps.unsqueeze(1), data["segmentation"]), dloss(pd, data["depth"])
    (lc + ls + ld).backward()
    rgrad = dict(ref.named_parameters())
    gkeys_e = [k for k, v in rgrad.items() if v.grad is not None]
    fx = {"loss_control": np.float64(lc), "loss_seg": np.float64(ls), "loss_depth": np.float64(ld),
          "gnorm_all": np.array([float(rgrad[k].grad.double().norm()) for k in gkeys_e])}
    for k in probe:
        fx["gsample::" + k] = sample(rgrad[k].grad).numpy()
    np.savez_compressed(os.path.join(OUT, "model_evalgrad_b8.npz"), **fx)
    meta["model_evalgrad_b8"] = {"batch_seed": 11, "noise_seed": 11, "probe": probe,
                                 "grad_keys": gkeys_e, "sample": SAMPLE}
    ref.zero_grad(set_to_none=True)

    ref.load_state_dict(state)
    orc.load_state_dict(state)
    ref.train(), orc.train()
    with FixedRand(noise):
        pc, ps, pd = ref(data)
    lc, ls, ld = closs(pc, data), sloss(ps.unsqueeze(1), data["segmentation"]), dloss(pd, data["depth"])
    (lc + ls + ld).backward()
    rgrad = dict(ref.named_parameters())
    losses_o, _ = O.train_losses(orc, data, noise)
    losses_o["train_loss"].backward()
    ograd = dict(orc.named_parameters())
    lerr = {"control": abs(float(lc) - float(losses_o["control_loss"])),
            "seg": abs(float(ls) - float(losses_o["segmentation_loss"])),
            "depth": abs(float(ld) - float(losses_o["depth_loss"]))}
    gkeys = [k for k, v in rgrad.items() if v.grad is not None]
    gerr = {k: rel(ograd[k].grad, rgrad[k].grad) for k in gkeys}
    print("oracle vs reference, train B=8 losses:", lerr, "max grad rel:", max(gerr.values()))
    assert max(lerr.values()) < 1e-5 and max(gerr.values()) < 1e-5
    fx = {"loss_control": np.float64(lc), "loss_seg": np.float64(ls), "loss_depth": np.float64(ld),
          "pred_control": pc.detach().numpy(),
          "seg_sample": sample(ps).numpy(), "seg_norm": np.float64(ps.detach().double().norm()),
          "depth_sample": sample(pd).numpy(), "depth_norm": np.float64(pd.detach().double().norm()),
          "gnorm_all": np.array([float(rgrad[k].grad.double().norm()) for k in gkeys])}
    for k in probe:
        fx["gsample::" + k] = sample(rgrad[k].grad).numpy()
    np.savez_compressed(os.path.join(OUT, "model_train_b8.npz"), **fx)
    meta["model_train_b8"] = {"batch_seed": 11, "noise_seed": 11, "probe": probe,
                              "grad_keys": gkeys, "sample": SAMPLE,
                              "oracle_loss_abs_err": lerr,
                              "oracle_grad_rel_err_max": max(gerr.values())}


def b8_bf16amp_fixtures(ref, state, closs, sloss, dloss, meta):
    """C3 comparator: the reference's own deterministic-train step at the B=8 bench batch run
    the way a bf16 mixed-precision trainer runs the modules the product's C3 mode puts on bf16
    operands — the camera encoder, BEV encoder and segmentation head (conv GEMMs) and, since
    round 3, the feature-fusion encoder and control decoder (their linear / attention
    projections) — their forward under torch.autocast(bfloat16) (the CPU autocast; its bf16
    op list covers conv / linear / matmul like the GPU one), fp32 parameters and gradients;
    lift-splat, the depth softmax and the losses stay fp32 as in the product.  Its error
    against the fp64 oracle is the bf16 error budget the product's C3 mode is held to
    (tests/test_train_step_b8_gpu.py)."""
    data = synthetic.synthetic_batch(8, seed=11)
    noise = synthetic.target_noise(8, seed=11)
    deterministic(ref)
    ref.load_state_dict(state)
    ref.train()
    ref.zero_grad(set_to_none=True)
    # the bf16 modules run under autocast; their outputs return to fp32 at the module boundary
    # (the reference's lift-splat index_put and everything after it require fp32: the whole
    # model under autocast raises in model/bev_model.py:103)
    conv_mods = (ref.bev_model.cam_encoder, ref.bev_encoder, ref.segmentation_head,
                 ref.feature_fusion, ref.control_predict)
    saved = [m.forward for m in conv_mods]

    def amp(fwd):
        def run(*a, **k):
            with torch.autocast("cpu", dtype=torch.bfloat16):
                out = fwd(*a, **k)
            if isinstance(out, tuple):
                return tuple(o.float() for o in out)
            return out.float()
        return run

    for m in conv_mods:
        m.forward = amp(m.forward)
    try:
        with FixedRand(noise):
            pc, ps, pd = ref(data)
    finally:
        for m, f in zip(conv_mods, saved):
            m.forward = f
    lc, ls, ld = closs(pc, data), sloss(ps.unsqueeze(1), data["segmentation"]), dloss(pd, data["depth"])
    (lc + ls + ld).backward()
    rgrad = dict(ref.named_parameters())
    gkeys = meta["model_train_b8"]["grad_keys"]
    assert [k for k, v in rgrad.items() if v.grad is not None] == gkeys
    fx = {"loss_control": np.float64(lc.float()), "loss_seg": np.float64(ls.float()),
          "loss_depth": np.float64(ld.float()),
          "pred_control": pc.detach().float().numpy(),
          "seg_sample": sample(ps.float()).numpy(), "depth_sample": sample(pd.float()).numpy(),
          "gnorm_all": np.array([float(rgrad[k].grad.double().norm()) for k in gkeys])}
    for k in meta["model_train_b8"]["probe"]:
        fx["gsample::" + k] = sample(rgrad[k].grad).numpy()
    np.savez_compressed(os.path.join(OUT, "model_train_b8_bf16amp.npz"), **fx)
    meta["model_train_b8_bf16amp"] = {"batch_seed": 11, "noise_seed": 11,
                                      "autocast": "cpu bfloat16: cam_encoder, bev_encoder, segmentation_head, "
                                                  "feature_fusion, control_predict forward",
                                      "grad_keys": "model_train_b8"}
    ref.zero_grad(set_to_none=True)


def c4_fixtures(cfg, meta):
    """BASELINE configs[3] (C4: 6 cameras at 512x512, B=1) through the full reference model:
    eval forward + predict, and one deterministic-train forward/backward (losses, output
    slices, probed gradient norms).  The oracle must reproduce the reference first."""
    from model.parking_model import ParkingModel
    from loss.control_loss import ControlLoss
    from loss.seg_loss import SegmentationLoss
    from loss.depth_loss import DepthLoss
    cfg.final_dim = [512, 512]
    cfg.image_crop = 512
    torch.manual_seed(0)
    ref = ParkingModel(cfg)
    state = make_state(ref.state_dict(), seed=1234)
    ref.load_state_dict(state)

    class CfgC4(O.Cfg):
        final_dim = [512, 512]

    orc = O.ParkingModelRef(CfgC4, dropout=False)
    orc.load_state_dict(state)
    data = synthetic.synthetic_batch(1, seed=13, hires=True)
    noise = synthetic.target_noise(1, seed=13)
    ref.eval(), orc.eval()
    with torch.no_grad(), FixedRand(noise):
        pc, ps, pd = ref(data)
        tok, _, _, tgt = ref.predict({**data, "gt_control": data["gt_control"][:, :1]})
    with torch.no_grad():
        qc, qs, qd = orc(data, noise)
    errs = {"control": rel(qc, pc), "seg": rel(qs, ps), "depth": rel(qd, pd)}
    print("C4 oracle vs reference, eval:", errs)
    assert max(errs.values()) < 1e-6
    np.savez_compressed(os.path.join(OUT, "model_eval_c4.npz"), pred_control=pc.numpy(),
                        pred_segmentation=ps.numpy(), pred_depth=pd.numpy(), predict_tokens=tok.numpy(),
                        bev_target=tgt.numpy())
    meta["model_eval_c4"] = {"batch_seed": 13, "noise_seed": 13, "hires": True, "oracle_rel_err": errs}

    deterministic(ref)
    closs, dloss = ControlLoss(cfg), DepthLoss(cfg)
    sloss = SegmentationLoss(class_weights=torch.Tensor(cfg.seg_vehicle_weights))
    # eval-mode gradients (BN on running statistics): the well-conditioned full backward
    ref.load_state_dict(state)
    ref.eval()
    with FixedRand(noise):
        pc, ps, pd = ref(data)
    lc, ls, ld = closs(pc, data), sloss(ps.unsqueeze(1), data["segmentation"]), dloss(pd, data["depth"])
    (lc + ls + ld).backward()
    rgrad = dict(ref.named_parameters())
    gkeys_e = [k for k, v in rgrad.items() if v.grad is not None]
    np.savez_compressed(os.path.join(OUT, "model_evalgrad_c4.npz"),
                        loss_control=np.float64(lc), loss_seg=np.float64(ls), loss_depth=np.float64(ld),
                        gnorm_all=np.array([float(rgrad[k].grad.double().norm()) for k in gkeys_e]))
    meta["model_evalgrad_c4"] = {"batch_seed": 13, "noise_seed": 13, "hires": True, "grad_keys": gkeys_e}
    ref.zero_grad(set_to_none=True)
    # deterministic train (BN batch statistics over 6 cameras)
    ref.load_state_dict(state)
    ref.train()
    with FixedRand(noise):
        pc, ps, pd = ref(data)
    lc, ls, ld = closs(pc, data), sloss(ps.unsqueeze(1), data["segmentation"]), dloss(pd, data["depth"])
    (lc + ls + ld).backward()
    rgrad = dict(ref.named_parameters())
    gkeys = [k for k, v in rgrad.items() if v.grad is not None]
    fx = {"loss_control": np.float64(lc), "loss_seg": np.float64(ls), "loss_depth": np.float64(ld),
          "pred_control": pc.detach().numpy(),
          "seg_slice": ps.detach()[:, :, 90:110, 90:110].numpy(),
          "depth_slice": pd.detach()[:, :, 10:14].numpy(),
          "gnorm_all": np.array([float(rgrad[k].grad.double().norm()) for k in gkeys])}
    np.savez_compressed(os.path.join(OUT, "model_train_c4.npz"), **fx)
    meta["model_train_c4"] = {"batch_seed": 13, "noise_seed": 13, "hires": True, "grad_keys": gkeys}


def c4b4_fixtures(cfg, meta):
    """The benched C4 step's batch shape (BASELINE configs[3]: 6 cameras at 512x512, B=4 per
    GPU): one deterministic-train forward/backward of the reference (BN batch statistics over
    24 camera images / 4 BEV samples), its three losses, control logits, every parameter's
    gradient norm and strided samples of the probe tensors' gradients.  The captured B=4 C4
    TrainStep is held to it (tests/test_model_c4_gpu.py)."""
    from model.parking_model import ParkingModel
    from loss.control_loss import ControlLoss
    from loss.seg_loss import SegmentationLoss
    from loss.depth_loss import DepthLoss
    cfg.final_dim = [512, 512]
    cfg.image_crop = 512
    torch.manual_seed(0)
    ref = ParkingModel(cfg)
    state = make_state(ref.state_dict(), seed=1234)
    deterministic(ref)
    ref.load_state_dict(state)
    ref.train()
    data = synthetic.synthetic_batch(4, seed=17, hires=True)
    noise = synthetic.target_noise(4, seed=17)
    closs, dloss = ControlLoss(cfg), DepthLoss(cfg)
    sloss = SegmentationLoss(class_weights=torch.Tensor(cfg.seg_vehicle_weights))
    with FixedRand(noise):
        pc, ps, pd = ref(data)
    lc, ls, ld = closs(pc, data), sloss(ps.unsqueeze(1), data["segmentation"]), dloss(pd, data["depth"])
    (lc + ls + ld).backward()
    rgrad = dict(ref.named_parameters())
    gkeys = [k for k, v in rgrad.items() if v.grad is not None]
    probe = make_grad_probe_keys(state.keys())
    fx = {"loss_control": np.float64(lc), "loss_seg": np.float64(ls), "loss_depth": np.float64(ld),
          "pred_control": pc.detach().numpy(),
          "seg_sample": sample(ps).numpy(), "depth_sample": sample(pd).numpy(),
          "gnorm_all": np.array([float(rgrad[k].grad.double().norm()) for k in gkeys])}
    for k in probe:
        fx["gsample::" + k] = sample(rgrad[k].grad).numpy()
    np.savez_compressed(os.path.join(OUT, "model_train_c4b4.npz"), **fx)
    meta["model_train_c4b4"] = {"batch_seed": 17, "noise_seed": 17, "hires": True, "batch": 4,
                                "probe": probe, "grad_keys": gkeys, "sample": SAMPLE}


def main(only=None):
    install_shims()
    torch.set_num_threads(8)
    import yaml
    from tool.config import get_cfg
    from model.parking_model import ParkingModel
    from model.bev_model import BevModel
    from loss.control_loss import ControlLoss
    from loss.seg_loss import SegmentationLoss
    from loss.depth_loss import DepthLoss

    with open(os.path.join(REF, "config", "training.yaml")) as f:
        cfg = get_cfg(yaml.safe_load(f))
    cfg.device = torch.device("cpu")
    meta = {"generator": "tests/golden/make_golden.py", "reference": REF,
            "torch": torch.__version__, "weights_seed": 1234}
    if only in ("c4", "c4b4"):  # add the C4 fixtures, keep the others and their meta
        with open(os.path.join(OUT, "meta.json")) as f:
            meta = json.load(f)
        (c4_fixtures if only == "c4" else c4b4_fixtures)(cfg, meta)
        with open(os.path.join(OUT, "meta.json"), "w") as f:
            json.dump(meta, f, indent=1)
        print("wrote C4 golden vectors to", OUT)
        return
    if only == "b8bf16":  # add the C3 (bf16 autocast) comparator, keep everything else
        with open(os.path.join(OUT, "meta.json")) as f:
            meta = json.load(f)
        torch.manual_seed(0)
        ref = ParkingModel(cfg)
        state = make_state(ref.state_dict(), seed=1234)
        b8_bf16amp_fixtures(ref, state, ControlLoss(cfg),
                            SegmentationLoss(class_weights=torch.Tensor(cfg.seg_vehicle_weights)),
                            DepthLoss(cfg), meta)
        with open(os.path.join(OUT, "meta.json"), "w") as f:
            json.dump(meta, f, indent=1)
        print("wrote the B=8 bf16-autocast comparator to", OUT)
        return
    if only == "b8":  # regenerate only the B=8 fixtures, keep the others and their meta
        with open(os.path.join(OUT, "meta.json")) as f:
            meta = json.load(f)
        torch.manual_seed(0)
        ref = ParkingModel(cfg)
        state = make_state(ref.state_dict(), seed=1234)
        orc = O.ParkingModelRef(O.Cfg, dropout=False)
        b8_fixtures(ref, orc, state, cfg, ControlLoss(cfg),
                    SegmentationLoss(class_weights=torch.Tensor(cfg.seg_vehicle_weights)),
                    DepthLoss(cfg), meta)
        with open(os.path.join(OUT, "meta.json"), "w") as f:
            json.dump(meta, f, indent=1)
        print("wrote B=8 golden vectors to", OUT)
        return

    # ---------------- (1) geometry / integer pillar index (model/bev_model.py:45-96) ----
    torch.manual_seed(0)
    ref = ParkingModel(cfg)
    bm = ref.bev_model
    K, E = synthetic.rig(4, 256)
    Kb, Eb = K.unsqueeze(0), E.unsqueeze(0)
    xyz = bm.get_geometry(Kb, Eb)
    res, start, dim = bm.bev_res.data, bm.bev_start_pos.data, bm.bev_dim.data
    pillar = O.pillar_index(xyz, res, start, dim).to(torch.int32)
    # same computation through the reference's own expressions (bev_model.py:85-95)
    g = ((xyz[0] - (start - res / 2.0)) / res).view(-1, 3).long()
    keep = ((g[:, 0] >= 0) & (g[:, 0] < dim[0]) & (g[:, 1] >= 0) & (g[:, 1] < dim[1])
            & (g[:, 2] >= 0) & (g[:, 2] < dim[2]))
    rk = g[:, 0] * (dim[1] * dim[2]) + g[:, 1] * dim[2] + g[:, 2]
    assert torch.equal(pillar.view(-1).long()[keep], rk[keep]) and (pillar.view(-1)[~keep] == -1).all()
    xo = O.geometry(bm.frustum.data, Kb, Eb)
    assert torch.equal(xo, xyz), "oracle geometry must be bitwise identical to the reference"
    comb, trans = O.rig_transforms(Kb, Eb)
    lo = (start - res / 2.0)
    np.savez_compressed(os.path.join(OUT, "geometry_4cam_256.npz"),
                        K=K.numpy(), E=E.numpy(), combine=comb[0].numpy(), trans=trans[0].numpy(),
                        frustum=bm.frustum.data.numpy(), lo=lo.numpy(), res=res.numpy(),
                        dim=dim.numpy(), pillar=pillar[0].numpy(), xyz=xyz[0].numpy())
    meta["geometry_4cam_256"] = {"kept": int(keep.sum()), "unique": int(rk[keep].unique().numel())}

    # hi-res 6-cam 512^2 rig (C4): store the table hash, not the table
    K6, E6 = synthetic.rig(6, 512, 512, 512)
    hb = BevModel.__new__(BevModel)
    torch.nn.Module.__init__(hb)
    hb.cfg = types.SimpleNamespace(final_dim=[512, 512], d_bound=cfg.d_bound)
    hb.down_sample = 8
    hb.frustum = hb.create_frustum()
    xyz6 = hb.get_geometry(K6.unsqueeze(0), E6.unsqueeze(0))
    p6 = O.pillar_index(xyz6, res, start, dim).to(torch.int32)[0].contiguous()
    assert torch.equal(O.geometry(hb.frustum.data, K6.unsqueeze(0), E6.unsqueeze(0)), xyz6)
    c6, t6 = O.rig_transforms(K6.unsqueeze(0), E6.unsqueeze(0))
    np.savez_compressed(os.path.join(OUT, "geometry_6cam_512.npz"), K=K6.numpy(), E=E6.numpy(),
                        combine=c6[0].numpy(), trans=t6[0].numpy(), frustum=hb.frustum.data.numpy())
    meta["geometry_6cam_512"] = {"pillar_sha256": hashlib.sha256(p6.numpy().tobytes()).hexdigest(),
                                 "kept": int((p6 >= 0).sum()),
                                 "unique": int(p6[p6 >= 0].unique().numel())}

    # ---------------- (2) lift-splat fwd/bwd at reduced channels (bev_model.py:59-107) ----
    B, N, D, h, w, C = 1, 4, 48, 32, 32, 4
    gl = torch.Generator().manual_seed(7)
    logits = torch.randn(B * N, D, h, w, generator=gl) * 2.0
    feat = torch.randn(B * N, C, h, w, generator=gl)
    gout = torch.randn(B, C, 200, 200, generator=gl)
    prob = logits.softmax(1).requires_grad_(True)
    featr = feat.clone().requires_grad_(True)
    outer = prob.unsqueeze(1) * featr.unsqueeze(2)
    outer = outer.view(B, N, *outer.shape[1:]).permute(0, 1, 3, 4, 5, 2)
    bev = bm.proj_bev_feature(xyz, outer)
    bev.backward(gout)
    prob_o = logits.softmax(1).requires_grad_(True)
    feat_o = feat.clone().requires_grad_(True)
    outer_o = (prob_o.unsqueeze(1) * feat_o.unsqueeze(2)).view(B, N, C, D, h, w).permute(0, 1, 3, 4, 5, 2)
    bev_o = O.splat(xyz, outer_o, res, start, dim)
    bev_o.backward(gout)
    assert torch.equal(bev_o, bev) and torch.equal(prob_o.grad, prob.grad) and torch.equal(feat_o.grad, featr.grad)
    np.savez_compressed(os.path.join(OUT, "lss_c4.npz"), bev=bev.detach().numpy(),
                        grad_prob=prob.grad.numpy(), grad_feat=featr.grad.numpy())
    meta["lss_c4"] = {"seed": 7, "shape": [B, N, D, h, w, C], "logit_scale": 2.0}

    # ---------------- (3) full model, closed-form weights -----------------------------
    state = make_state(ref.state_dict(), seed=1234)
    ref.load_state_dict(state)
    orc = O.ParkingModelRef(O.Cfg, dropout=False)
    assert list(orc.state_dict().keys()) == list(ref.state_dict().keys())
    orc.load_state_dict(state)
    meta["state_keys"] = [[k, list(v.shape), str(v.dtype)] for k, v in ref.state_dict().items()]

    closs = ControlLoss(cfg)
    sloss = SegmentationLoss(class_weights=torch.Tensor(cfg.seg_vehicle_weights))
    dloss = DepthLoss(cfg)

    # (3a) eval forward + predict, B=1
    data = synthetic.synthetic_batch(1, seed=3)
    noise = synthetic.target_noise(1, seed=3)
    ref.eval(), orc.eval()
    with torch.no_grad(), FixedRand(noise):
        pc, ps, pd = ref(data)
        tok, ps2, pd2, tgt = ref.predict({**data, "gt_control": data["gt_control"][:, :1]})
    with torch.no_grad():
        qc, qs, qd = orc(data, noise)
        qtok, _, _, qtgt = orc.predict({**data, "gt_control": data["gt_control"][:, :1]}, noise)
    errs = {"control": rel(qc, pc), "seg": rel(qs, ps), "depth": rel(qd, pd)}
    print("oracle vs reference, eval:", errs)
    assert max(errs.values()) < 1e-6 and torch.equal(qtok, tok) and torch.equal(qtgt, tgt)
    np.savez_compressed(os.path.join(OUT, "model_eval_b1.npz"), pred_control=pc.numpy(),
                        pred_segmentation=ps.numpy(), pred_depth=pd.numpy(), predict_tokens=tok.numpy(),
                        bev_target=tgt.numpy())
    meta["model_eval_b1"] = {"batch_seed": 3, "noise_seed": 3, "oracle_rel_err": errs}

    # (3b) deterministic-train forward/backward, B=2
    deterministic(ref)
    ref.load_state_dict(state)
    orc.load_state_dict(state)
    ref.train(), orc.train()
    data = synthetic.synthetic_batch(2, seed=5)
    noise = synthetic.target_noise(2, seed=5)
    probe = make_grad_probe_keys(state.keys())
    with FixedRand(noise):
        pc, ps, pd = ref(data)
    lc, ls, ld = closs(pc, data), sloss(ps.unsqueeze(1), data["segmentation"]), dloss(pd, data["depth"])
    (lc + ls + ld).backward()
    rgrad = dict(ref.named_parameters())
    losses_o, (qc, qs, qd) = O.train_losses(orc, data, noise)
    losses_o["train_loss"].backward()
    ograd = dict(orc.named_parameters())
    lerr = {"control": abs(float(lc) - float(losses_o["control_loss"])),
            "seg": abs(float(ls) - float(losses_o["segmentation_loss"])),
            "depth": abs(float(ld) - float(losses_o["depth_loss"]))}
    gerr = {k: rel(ograd[k].grad, rgrad[k].grad) for k in probe}
    print("oracle vs reference, train losses:", lerr)
    print("oracle vs reference, grads:", max(gerr.values()))
    assert max(lerr.values()) < 1e-5 and max(gerr.values()) < 1e-5
    fx = {"loss_control": np.float64(lc), "loss_seg": np.float64(ls), "loss_depth": np.float64(ld),
          "pred_control": pc.detach().numpy(),
          "seg_norm": np.float64(ps.detach().double().norm()), "seg_slice": ps.detach()[:, :, 90:110, 90:110].numpy(),
          "depth_norm": np.float64(pd.detach().double().norm()), "depth_slice": pd.detach()[:, :, 10:14].numpy()}
    for k in probe:
        gk = rgrad[k].grad.reshape(-1)
        fx["gnorm::" + k] = np.float64(gk.double().norm())
        fx["gslice::" + k] = gk[:4096].numpy()
    np.savez_compressed(os.path.join(OUT, "model_train_b2.npz"), **fx)
    meta["model_train_b2"] = {"batch_seed": 5, "noise_seed": 5, "probe": probe,
                              "oracle_loss_abs_err": lerr, "oracle_grad_rel_err_max": max(gerr.values())}

    # (3c/3d) the C2 bench batch, B=8 (eval and deterministic-train)
    b8_fixtures(ref, orc, state, cfg, closs, sloss, dloss, meta)

    with open(os.path.join(OUT, "meta.json"), "w") as f:
        json.dump(meta, f, indent=1)
    print("wrote golden vectors to", OUT)


if __name__ == "__main__":
    main(sys.argv[1] if len(sys.argv) > 1 else None)
