"""Drop-in API checks that need no GPU: state-dict layout, checkpoint loading, config."""
import os

import torch

from helpers import meta


def _cfg(**kw):
    from tool.config import default_cfg
    return default_cfg(**kw)


def test_state_dict_keys_shapes_dtypes_match_reference():
    from model.parking_model import ParkingModel
    sd = ParkingModel(_cfg()).state_dict()
    ref = meta()["state_keys"]
    assert [k for k, _, _ in ref] == list(sd.keys())
    for k, shape, dtype in ref:
        assert list(sd[k].shape) == shape and str(sd[k].dtype) == dtype, k


def test_loads_reference_checkpoint_layout(tmp_path):
    """agent/parking_agent.py:257-264: ckpt['state_dict'] with the 'parking_model.' prefix."""
    from collections import OrderedDict
    from model.parking_model import ParkingModel
    from trainer.pl_trainer import ParkingTrainingModule
    mod = ParkingTrainingModule(_cfg())
    path = os.path.join(tmp_path, "last.ckpt")
    torch.save({"state_dict": mod.state_dict(), "epoch": 0}, path)
    ckpt = torch.load(path, map_location="cpu", weights_only=True)
    sd = OrderedDict((k.replace("parking_model.", ""), v) for k, v in ckpt["state_dict"].items())
    m = ParkingModel(_cfg())
    m.load_state_dict(sd)  # strict
    assert all(k.startswith("parking_model.") for k in ckpt["state_dict"])


def test_config_mirrors_reference_yaml():
    c = _cfg()
    assert c.bev_x_bound == [-10.0, 10.0, 0.1] and c.d_bound == [0.5, 12.5, 0.25]
    assert c.tf_en_dim == 258 and c.tf_de_tgt_dim == 15 and c.token_nums == 204


def test_frustum_and_bev_params_identical_to_oracle():
    from model.parking_model import ParkingModel
    from oracle import parking_ref as O
    m = ParkingModel(_cfg())
    fr = O.frustum([256, 256], 8, [0.5, 12.5, 0.25])
    assert torch.equal(m.bev_model.frustum.data, fr)
    res, start, dim = O.bev_params([-10.0, 10.0, 0.1], [-10.0, 10.0, 0.1], [-10.0, 10.0, 20.0])
    assert torch.equal(m.bev_model.bev_res.data, res) and torch.equal(m.bev_model.bev_dim.data, dim)
    assert torch.equal(m.bev_model.bev_start_pos.data, start)


def test_layer4_unused_and_parameter_count():
    from model.parking_model import ParkingModel
    m = ParkingModel(_cfg())
    total = sum(p.numel() for p in m.parameters())
    assert total == 28134708


def test_pl_format_checkpoint_round_trip(tmp_path):
    """PL-1.5-format .ckpt written without PL (trainer/pl_trainer.py:17-22,39), read back with
    the restricted unpickler: weights (parking_model.* keys), hyper_parameters['cfg'] as a
    tool.config.Configuration, Adam + CosineAnnealingLR state; the agent's load path
    (agent/parking_agent.py:257-264) builds the model from it strictly."""
    from e2ep_amd import checkpoint
    from tool.config import Configuration
    from trainer.pl_trainer import ParkingTrainingModule
    torch.manual_seed(0)
    mod = ParkingTrainingModule(_cfg())
    opt_d = mod.configure_optimizers()
    opt, sched = opt_d["optimizer"], opt_d["lr_scheduler"]
    # one fake step so the Adam state is populated
    for p in list(mod.parameters())[:5]:
        p.grad = torch.ones_like(p)
    opt.step()
    sched.step()
    path = os.path.join(tmp_path, "E2EParking-epoch=00-val_loss=1.00.ckpt")
    cb = {"ModelCheckpoint{'monitor': 'val_loss', 'mode': 'min'}": {"best_model_score": torch.tensor(1.0),
                                                                     "best_model_path": path}}
    checkpoint.save_checkpoint(path, mod, opt, sched, epoch=3, global_step=42, callbacks=cb)
    ck = checkpoint.load_checkpoint(path)
    assert ck["epoch"] == 3 and ck["global_step"] == 42
    assert ck["pytorch-lightning_version"] == checkpoint.PL_VERSION
    cfg = ck["hyper_parameters"]["cfg"]
    assert isinstance(cfg, Configuration) and cfg.d_bound == mod.cfg.d_bound
    assert list(ck["state_dict"]) == list(mod.state_dict())
    assert all(k.startswith("parking_model.") for k in ck["state_dict"])
    m = checkpoint.load_parking_model(path)
    for (k, v), (k2, v2) in zip(m.state_dict().items(), mod.parking_model.state_dict().items()):
        assert k == k2 and torch.equal(v, v2)
    assert not m.training
    # resume: optimizer / scheduler state restored
    mod2 = ParkingTrainingModule(_cfg())
    d2 = mod2.configure_optimizers()
    ep, gs = checkpoint.restore_training(ck, mod2, d2["optimizer"], d2["lr_scheduler"])
    assert (ep, gs) == (3, 42)
    assert d2["lr_scheduler"].last_epoch == sched.last_epoch
    s1, s2 = opt.state_dict()["state"], d2["optimizer"].state_dict()["state"]
    assert s1.keys() == s2.keys() and all(torch.equal(s1[i]["exp_avg"], s2[i]["exp_avg"]) for i in s1)


def test_checkpoint_loader_rejects_foreign_pickles(tmp_path):
    """Only tool.config.Configuration / torch.device (and torch's own weights-only types) may be
    unpickled: any other class (here one defined in this test, standing in for arbitrary code)
    is refused."""
    import pickle
    import pytest
    from e2ep_amd import checkpoint
    path = os.path.join(tmp_path, "bad.ckpt")
    torch.save({"state_dict": {}, "hyper_parameters": {"x": _Foreign()}}, path)
    with pytest.raises(pickle.UnpicklingError):
        checkpoint.load_checkpoint(path)


class _Foreign:
    def __init__(self):
        self.payload = "not a Configuration"
