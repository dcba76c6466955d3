"""Closed-form, host-independent ParkingModel weights for parity tests (test infrastructure).

`make_state(template, seed)` fills every floating tensor of a state-dict template from a
CPU torch.Generator seeded once and walked in sorted key order, so the reference (golden
generation, this container), the oracle and the product (GPU box) all see identical
weights without shipping 112 MB of parameters.  Constants that define the geometry
(bev_res, bev_start_pos, bev_dim, frustum) and integer buffers keep their template values.

Scales keep activations O(1) through the net and make every BN affine non-trivial
(SURVEY.md §7 hard part 7: torchvision's zero_init_residual would otherwise hide every
BasicBlock conv2).
"""
import math

import torch

KEEP = ("bev_model.bev_res", "bev_model.bev_start_pos", "bev_model.bev_dim", "bev_model.frustum")


def make_state(template, seed=1234):
    g = torch.Generator().manual_seed(seed)
    out = {}
    for k in sorted(template):
        t = template[k]
        if k in KEEP or not t.is_floating_point():
            out[k] = t.clone()
            continue
        shape = t.shape
        if k.endswith("running_var"):
            v = 0.5 + torch.rand(shape, generator=g)
        elif k.endswith("running_mean"):
            v = 0.1 * torch.randn(shape, generator=g)
        elif "pos_embed" in k:
            v = 0.02 * torch.randn(shape, generator=g)
        elif t.dim() == 1 and k.endswith("weight"):
            v = 1.0 + 0.1 * torch.randn(shape, generator=g)
        elif t.dim() == 1:  # biases
            v = 0.05 * torch.randn(shape, generator=g)
        else:
            fan_in = max(1, math.prod(shape[1:]))
            v = torch.randn(shape, generator=g) * (1.0 / math.sqrt(fan_in))
        out[k] = v.to(t.dtype)
    return {k: out[k] for k in template}


def make_grad_probe_keys(keys):
    """A fixed, spread-out subset of parameter names whose gradients the fixtures record."""
    want = [
        "bev_model.cam_encoder.backbone._conv_stem.weight",
        "bev_model.cam_encoder.backbone._blocks.5._depthwise_conv.weight",
        "bev_model.cam_encoder.feature_layer_2.conv.3.weight",
        "bev_model.cam_encoder.depth_layer_2.conv.3.weight",
        "bev_model.cam_encoder.depth_layer_1.0.convs.1.0.weight",
        "bev_encoder.conv1.weight",
        "bev_encoder.layer1.0.conv2.weight",
        "bev_encoder.layer3.1.bn2.weight",
        "feature_fusion.tf_encoder.layers.0.self_attn.in_proj_weight",
        "feature_fusion.motion_encoder.0.weight",
        "control_predict.tf_decoder.layers.3.multihead_attn.in_proj_weight",
        "control_predict.output.weight",
        "segmentation_head.segmentation_head.0.weight",
        "segmentation_head.c5_conv.weight",
    ]
    return [k for k in want if k in keys]
