"""Configuration bag — same API as the reference's tool/config.py:7-111.

`Configuration` holds the YAML keys as attributes; `get_cfg(yaml_dict)` fills one from the
`parking_model` section.  The device defaults to the HIP device (`cuda` on PyTorch-ROCm).
Optional MI355X keys (absent from reference configs, defaults shown):
  deterministic: False   zero every dropout / drop-connect (SURVEY.md §8c protocol)
"""
import os
from datetime import datetime

import torch

_KEYS = [
    "log_every_n_steps", "check_val_every_n_epoch", "epochs", "learning_rate", "weight_decay",
    "batch_size", "training_map", "validation_map", "future_frame_nums", "hist_frame_nums",
    "token_nums", "image_crop", "bev_encoder_in_channel", "bev_encoder_out_channel",
    "bev_x_bound", "bev_y_bound", "bev_z_bound", "d_bound", "final_dim", "bev_down_sample",
    "use_depth_distribution", "backbone", "seg_classes", "seg_vehicle_weights", "tf_en_dim",
    "tf_en_heads", "tf_en_layers", "tf_en_dropout", "tf_en_bev_length", "tf_en_motion_length",
    "tf_de_dim", "tf_de_heads", "tf_de_layers", "tf_de_dropout", "tf_de_tgt_dim",
]


class Configuration:
    device = torch.device("cuda" if torch.cuda.is_available() else "cpu")
    data_dir = None
    log_dir = None
    checkpoint_dir = None
    deterministic = False


for _k in _KEYS:
    setattr(Configuration, _k, None)


def get_cfg(cfg_yaml: dict) -> Configuration:
    section = cfg_yaml["parking_model"]
    cfg = Configuration()
    stamp = datetime.now().strftime("%Y_%-m_%-d_%-H_%-M_%-S")
    cfg.data_dir = section["data_dir"]
    cfg.log_dir = os.path.join(section["log_dir"], "exp_" + stamp)
    cfg.checkpoint_dir = os.path.join(section["checkpoint_dir"], "exp_" + stamp)
    for k in _KEYS:
        setattr(cfg, k, section[k])
    cfg.deterministic = bool(section.get("deterministic", False))
    return cfg


def default_cfg(**overrides) -> Configuration:
    """The shipped config/training.yaml, with attribute overrides."""
    import yaml

    here = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    with open(os.path.join(here, "config", "training.yaml")) as f:
        cfg = get_cfg(yaml.safe_load(f))
    for k, v in overrides.items():
        setattr(cfg, k, v)
    return cfg
