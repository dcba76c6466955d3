"""Operator layer of the ParkingModel hot path on MI355X.

Every model module calls these functions instead of torch.nn.functional.  Each one names
the HIP kernel family that implements it (libe2ep_hip.so, include/e2ep.h); the few that are
still MIOpen / hipBLASLt calls through PyTorch are listed in DESIGN.md §"Kernel coverage"
with the round they move to HIP.
"""
import torch
import torch.nn.functional as F

from . import _lib


def _pad4(pad):
    if isinstance(pad, int):
        return (pad, pad, pad, pad)
    if len(pad) == 2:
        return (pad[1], pad[1], pad[0], pad[0])
    return tuple(pad)


def conv2d(x, weight, bias=None, stride=1, padding=0, dilation=1, groups=1):
    """NCHW convolution; padding is an int, (ph, pw) or (left, right, top, bottom)."""
    l, r, t, b = _pad4(padding)
    if l == r and t == b:
        return F.conv2d(x, weight, bias, stride, (t, l), dilation, groups)
    return F.conv2d(F.pad(x, (l, r, t, b)), weight, bias, stride, 0, dilation, groups)


def _act(x, act):
    if act is None:
        return x
    if act == "relu":
        return F.relu(x)
    if act == "swish":
        return x * torch.sigmoid(x)
    raise ValueError(act)


def bn_act(x, bn, act=None):
    """BatchNorm2d (train: batch statistics + running-stat update; eval: running stats) + act."""
    if bn.training and bn.track_running_stats and bn.num_batches_tracked is not None:
        bn.num_batches_tracked.add_(1)
    y = F.batch_norm(x, bn.running_mean, bn.running_var, bn.weight, bn.bias,
                     bn.training or not bn.track_running_stats, bn.momentum, bn.eps)
    return _act(y, act)


def squeeze_excite(x, reduce, expand):
    g = F.adaptive_avg_pool2d(x, 1)
    g = conv2d(g, reduce.weight, reduce.bias)
    g = conv2d(g * torch.sigmoid(g), expand.weight, expand.bias)
    return torch.sigmoid(g) * x


def drop_connect(x, p):
    keep = 1.0 - p
    mask = torch.floor(keep + torch.rand([x.shape[0], 1, 1, 1], dtype=x.dtype, device=x.device))
    return x / keep * mask


def upsample2x(x):
    return F.interpolate(x, scale_factor=2, mode="bilinear", align_corners=False)


def resize(x, size):
    return F.interpolate(x, size=size, mode="bilinear", align_corners=False)


def max_pool3s2(x):
    return F.max_pool2d(x, 3, 2, 1)


def lib_loaded():
    """True once libe2ep_hip.so is loaded (raises if it cannot be)."""
    _lib.load()
    return True
