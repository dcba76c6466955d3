"""Operator layer of the ParkingModel hot path on MI355X.

Model modules call these functions instead of torch.nn.functional; every one of them runs
an e2ep HIP kernel from libe2ep_hip.so (include/e2ep.h) — there is no PyTorch or CPU
fallback, and a missing library raises.  What still runs as PyTorch work is listed in
DESIGN.md §4: the token embedding and small elementwise glue (concat, a few autograd
accumulation adds); every GEMM, including the transformer linears, is an e2ep kernel.
"""
from . import conv as _conv
from . import nn_ops


def _pad4(pad):
    if isinstance(pad, int):
        return (pad, pad, pad, pad)
    if len(pad) == 2:  # (ph, pw) torch convention
        return (pad[1], pad[1], pad[0], pad[0])
    return tuple(pad)


def _pair(v):
    return (v, v) if isinstance(v, int) else tuple(v)


def conv2d(x, weight, bias=None, stride=1, padding=0, dilation=1, groups=1, act=None, skip=False,
           bn_stats=False):
    """NCHW convolution; padding is an int, (ph, pw) or (left, right, top, bottom).
    groups == channels (depthwise) goes to the depthwise kernels, groups == 1 to the
    implicit-GEMM MFMA kernels; act None | 'relu' is fused into the GEMM epilogue.
    skip=True (groups == 1): returns (y, x_skip), see e2ep_amd.conv.conv2d.
    bn_stats=True: a training BatchNorm follows; see e2ep_amd.conv.conv2d."""
    pad = _pad4(padding)
    if groups == 1:
        return _conv.conv2d(x, weight, bias, _pair(stride), pad, _pair(dilation),
                            nn_ops.ACT[act], skip=skip, bn_stats=bn_stats)
    assert not skip, "skip passthrough is for groups == 1 convs"
    if groups == x.shape[1] and weight.shape[0] == groups and weight.shape[1] == 1 and bias is None \
            and _pair(dilation) == (1, 1) and act is None:
        s = _pair(stride)
        assert s[0] == s[1]
        return nn_ops.depthwise_conv2d(x, weight, s[0], pad, bn_stats=bn_stats)
    raise NotImplementedError(f"e2ep conv2d: groups={groups} not on the hot path")


def bn_act(x, bn, act=None, res=None, dc_rand=None, dc_keep=1.0):
    """BatchNorm2d (train: batch stats + running update; eval: running stats)
    [+ drop-connect] [+ res] + act."""
    return nn_ops.batch_norm_act(x, bn, act, res, dc_rand, dc_keep)


def bn_act_depthwise(x, bn, act, conv, bn_stats=False):
    """conv(bn_act(x, bn, act)) for a depthwise SameConv `conv`, fused: the BN + activation
    are applied while the depthwise kernel loads its input (MBConv _bn0 -> swish ->
    _depthwise_conv); the normalised activation tensor is never written.  bn_stats: a
    training BatchNorm reads the output next (see conv2d)."""
    s = _pair(conv.stride)
    assert s[0] == s[1] and conv.groups == x.shape[1] and conv.bias is None
    return nn_ops.bn_act_depthwise_conv2d(x, bn, act, conv.weight, s[0], _pad4(conv.same),
                                          bn_stats=bn_stats)


def activation(x, act):
    return nn_ops.activation(x, act)


def squeeze_excite(x, reduce, expand):
    """efficientnet-pytorch MBConv SE: x * sigmoid(expand(swish(reduce(avgpool(x))))), one
    fused op (e2ep_se_fwd / e2ep_se_bwd)."""
    return nn_ops.squeeze_excite(x, reduce.weight, reduce.bias, expand.weight, expand.bias)


def bn_swish_squeeze_excite(x, bn, reduce, expand):
    """squeeze_excite(bn_act(x, bn, 'swish'), reduce, expand) fused: BN + swish applied on
    load by the SE kernels; the activation tensor is never stored."""
    return nn_ops.bn_swish_squeeze_excite(x, bn, reduce.weight, reduce.bias, expand.weight,
                                          expand.bias)


def upsample2x(x):
    return nn_ops.resize(x, scale_factor=2)


def resize(x, size):
    return nn_ops.resize(x, size=tuple(size))


def max_pool3s2(x):
    return nn_ops.max_pool3s2(x)


def global_avg_pool(x):
    return nn_ops.global_avg_pool(x)
