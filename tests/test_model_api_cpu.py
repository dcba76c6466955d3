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
