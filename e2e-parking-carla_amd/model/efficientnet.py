"""EfficientNet-b4 camera trunk with efficientnet-pytorch 0.7.1's module/key layout.

The reference builds its camera encoder on `EfficientNet.from_pretrained('efficientnet-b4')`
(reference model/cam_encoder.py:4,17) and keeps blocks 0-21 (:42-58).  This module keeps the
same state-dict keys (`_conv_stem`, `_bn0`, `_blocks.i._expand_conv` ...) so reference
checkpoints load unchanged, and the same semantics: static SAME padding computed for the
nominal 380-pixel input, BN momentum 0.01 / eps 1e-3, swish, squeeze-excitation, identity
skip (with drop-connect in training) on repeat blocks only.  Forward runs on e2ep_amd ops.
"""
import math

import torch
from torch import nn

from e2ep_amd import nn_ops, ops, rng

# b0 base stages: (repeats, kernel, stride, expand, in, out); b4 scales width 1.4 / depth 1.8
_STAGES = [(1, 3, 1, 1, 32, 16), (2, 3, 2, 6, 16, 24), (2, 5, 2, 6, 24, 40), (3, 3, 2, 6, 40, 80),
           (3, 5, 1, 6, 80, 112), (4, 5, 2, 6, 112, 192), (1, 3, 1, 6, 192, 320)]
_VARIANTS = {"b4": (1.4, 1.8, 380), "b0": (1.0, 1.0, 224)}


def _filters(c, width):
    c *= width
    r = max(8, int(c + 4) // 8 * 8)
    return int(r + 8 if r < 0.9 * c else r)


def _same(size, k, s):
    o = math.ceil(size / s)
    p = max((o - 1) * s + k - size, 0)
    return (p // 2, p - p // 2, p // 2, p - p // 2)  # left, right, top, bottom


class SameConv(nn.Conv2d):
    """nn.Conv2d whose zero padding is fixed from the nominal image size (0.7.1 semantics)."""

    def __init__(self, cin, cout, k, stride=1, groups=1, bias=True, size=1):
        super().__init__(cin, cout, k, stride=stride, padding=0, groups=groups, bias=bias)
        self.same = _same(size, k, stride)

    def forward(self, x, bn_stats=False):
        """bn_stats: a training BatchNorm reads the output next (its statistics come from this
        conv's epilogue where the kernel takes them, e2ep_conv_fwd_stats)."""
        return ops.conv2d(x, self.weight, self.bias, self.stride, self.same, 1, self.groups,
                          bn_stats=bn_stats)

    def forward_skip(self, x, bn_stats=False):
        """(conv(x), x_skip): x_skip feeds the block's skip connection; its gradient is added
        inside this conv's data-gradient kernel (e2ep_conv_dgrad_acc)."""
        return ops.conv2d(x, self.weight, self.bias, self.stride, self.same, 1, self.groups, skip=True,
                          bn_stats=bn_stats)


class MBConv(nn.Module):
    def __init__(self, cin, cout, k, stride, expand, size, first):
        super().__init__()
        mid = cin * expand
        self.expand, self.k, self.stride = expand, k, stride
        self.skip = (not first) and cin == cout  # first block of a stage never skips
        if expand != 1:
            self._expand_conv = SameConv(cin, mid, 1, bias=False, size=size)
            self._bn0 = nn.BatchNorm2d(mid, momentum=0.01, eps=1e-3)
        self._depthwise_conv = SameConv(mid, mid, k, stride, groups=mid, bias=False, size=size)
        self._bn1 = nn.BatchNorm2d(mid, momentum=0.01, eps=1e-3)
        sq = max(1, int(cin * 0.25))
        self._se_reduce = SameConv(mid, sq, 1)
        self._se_expand = SameConv(sq, mid, 1)
        self._project_conv = SameConv(mid, cout, 1, bias=False, size=math.ceil(size / stride))
        self._bn2 = nn.BatchNorm2d(cout, momentum=0.01, eps=1e-3)

    def forward(self, x, drop_connect_rate=None, dc_rand=None, alias=False):
        """dc_rand: this block's per-sample uniform draws for drop-connect (training); drawn
        here when not given (efficientnet-pytorch draws torch.rand([N,1,1,1]) per block).
        alias=True (blocks with an expand conv): returns (out, x_alias), x_alias being the
        expand conv's skip alias of x for another consumer of x (a trunk endpoint)."""
        st = self.training  # BN statistics from the 1x1 convs' epilogues (training BN)
        if alias:
            assert self.expand != 1 and not self.skip
            e, xa = self._expand_conv.forward_skip(x, st)
            y = ops.bn_act_depthwise(e, self._bn0, "swish", self._depthwise_conv, st)
            y = ops.bn_swish_squeeze_excite(y, self._bn1, self._se_reduce, self._se_expand)
            return ops.bn_act(self._project_conv(y, st), self._bn2, None), xa
        if self.expand != 1:  # _bn0 + swish applied inside the depthwise conv's input load
            if self.skip and x.is_cuda:
                e, x = self._expand_conv.forward_skip(x, st)
            else:
                e = self._expand_conv(x, st)
            y = ops.bn_act_depthwise(e, self._bn0, "swish", self._depthwise_conv, st)
        elif self.skip and x.is_cuda:  # x feeds the depthwise conv and the skip (nn_ops.fork2)
            xd, x = nn_ops.fork2(x)
            y = self._depthwise_conv(xd, st)
        else:
            y = self._depthwise_conv(x, st)
        y = ops.bn_swish_squeeze_excite(y, self._bn1, self._se_reduce, self._se_expand)
        if not self.skip:
            return ops.bn_act(self._project_conv(y, st), self._bn2, None)
        if drop_connect_rate and self.training:
            # bn2 -> x / keep * floor(keep + u) -> + inputs, fused into the BN kernels
            if dc_rand is None:
                dc_rand = torch.rand(x.shape[0], dtype=x.dtype, device=x.device)
            return ops.bn_act(self._project_conv(y, st), self._bn2, None, res=x, dc_rand=dc_rand,
                              dc_keep=1.0 - drop_connect_rate)
        return ops.bn_act(self._project_conv(y, st), self._bn2, None, res=x)  # fused skip add


class EfficientNetTrunk(nn.Module):
    """The stem + first `keep_blocks` MBConv blocks of EfficientNet (b4: 22 blocks)."""

    def __init__(self, version="b4", keep_blocks=22, drop_connect_rate=0.2):
        super().__init__()
        width, depth, size = _VARIANTS[version]
        self.drop_connect_rate = drop_connect_rate
        stem = _filters(32, width)
        self._conv_stem = SameConv(3, stem, 3, 2, bias=False, size=size)
        self._bn0 = nn.BatchNorm2d(stem, momentum=0.01, eps=1e-3)
        size = math.ceil(size / 2)
        blocks = []
        for r, k, s, e, i, o in _STAGES:
            cin, cout = _filters(i, width), _filters(o, width)
            for j in range(int(math.ceil(depth * r))):
                blocks.append(MBConv(cin if j == 0 else cout, cout, k, s if j == 0 else 1, e, size, j == 0))
                if j == 0:
                    size = math.ceil(size / s)
        self._blocks = nn.ModuleList(blocks[:keep_blocks])

    def forward(self, x):
        """Returns the list of stride endpoints (reduction_1..) and the final map."""
        x = ops.bn_act(self._conv_stem(x), self._bn0, "swish")
        ends, prev = [], x
        n = len(self._blocks)
        # all blocks' drop-connect draws in one launch (one row of N per block)
        # (from the step's uniform pool, e2ep_amd.rng, inside a training forward)
        u = (rng.uniform((n, x.shape[0]), x.device, x.dtype)
             if self.training and self.drop_connect_rate else None)
        for i, blk in enumerate(self._blocks):
            dcr = self.drop_connect_rate * i / n if self.drop_connect_rate else None
            ui = None if u is None else u[i]
            if blk.stride > 1 and blk.expand != 1 and not blk.skip:
                # x is an endpoint and this block's input: the endpoint is the expand conv's
                # skip alias, so the two gradients of x meet in that conv's dgrad epilogue
                x, prev = blk(x, dcr, ui, alias=True)
            else:
                x = blk(x, dcr, ui)
            if prev.shape[2] > x.shape[2]:
                ends.append(prev)
            prev = x
        ends.append(x)
        return ends
