"""ORACLE / TEST INFRASTRUCTURE ONLY — never imported by the product package.

CPU restatement of the two third-party trunks the reference builds its ParkingModel on.
Neither package is installed in this image and both are absent from /root/reference, so
their published algorithms are restated here from the pinned versions:

* efficientnet-pytorch 0.7.1 (reference/environment.yml:107), used at
  reference/model/cam_encoder.py:4,17,42-58,65,69-73:
  - static "SAME" padding computed for the model's nominal image size (380 for b4),
    not for the actual 256x256 input;
  - BN momentum 1-0.99 = 0.01, eps 1e-3;
  - MBConv: [expand 1x1 + BN + swish] -> depthwise kxk + BN + swish -> SE(avgpool, 1x1,
    swish, 1x1, sigmoid gate) -> project 1x1 + BN -> [drop-connect + identity skip];
  - the skip is taken only by repeat blocks (decoded `stride` is the list [s] for the first
    block of a group, and `[1] == 1` is False in Python; repeats get the int 1).
* torchvision 0.14.1 (reference/environment.yml:91), used at
  reference/model/bev_encoder.py:5,11-21: resnet18(zero_init_residual=True).

Parity of these restatements against the real packages is UNPINNED (no fixture in the
reference covers them; the packages are not installed).  The golden-vector script injects
these modules under the third-party names so the reference's own code runs unmodified.
"""
import math
from collections import namedtuple

import torch
import torch.nn.functional as F
from torch import nn

# ----------------------------------------------------------------------------------------
# EfficientNet (efficientnet-pytorch 0.7.1 semantics)
# ----------------------------------------------------------------------------------------

_B4 = dict(width=1.4, depth=1.8, res=380, dropout=0.4)
_BLOCKS = [  # (repeats, kernel, stride, expand, in, out) of the b0 base network, se 0.25
    (1, 3, 1, 1, 32, 16),
    (2, 3, 2, 6, 16, 24),
    (2, 5, 2, 6, 24, 40),
    (3, 3, 2, 6, 40, 80),
    (3, 5, 1, 6, 80, 112),
    (4, 5, 2, 6, 112, 192),
    (1, 3, 1, 6, 192, 320),
]
_B0 = dict(width=1.0, depth=1.0, res=224, dropout=0.2)

GlobalParams = namedtuple("GlobalParams", ["width", "depth", "image_size", "dropout_rate",
                                           "drop_connect_rate", "bn_momentum", "bn_eps"])
BlockArgs = namedtuple("BlockArgs", ["repeats", "kernel", "stride", "expand", "inp", "out",
                                     "se_ratio", "id_skip"])


def round_filters(filters, width, divisor=8):
    filters *= width
    new = max(divisor, int(filters + divisor / 2) // divisor * divisor)
    if new < 0.9 * filters:
        new += divisor
    return int(new)


def round_repeats(repeats, depth):
    return int(math.ceil(depth * repeats))


def _same_pad(image_size, k, s, dilation=1):
    ih = iw = image_size
    oh, ow = math.ceil(ih / s), math.ceil(iw / s)
    ph = max((oh - 1) * s + (k - 1) * dilation + 1 - ih, 0)
    pw = max((ow - 1) * s + (k - 1) * dilation + 1 - iw, 0)
    return (pw // 2, pw - pw // 2, ph // 2, ph - ph // 2)


class StaticSameConv2d(nn.Conv2d):
    """Conv2d with the padding fixed at construction from a nominal image size."""

    def __init__(self, cin, cout, k, stride=1, groups=1, bias=True, image_size=None):
        super().__init__(cin, cout, k, stride=stride, padding=0, groups=groups, bias=bias)
        s = self.stride[0]
        self.pad = _same_pad(image_size, k, s) if image_size is not None else (0, 0, 0, 0)

    def forward(self, x):
        if any(self.pad):
            x = F.pad(x, self.pad)
        return F.conv2d(x, self.weight, self.bias, self.stride, 0, self.dilation, self.groups)


class Swish(nn.Module):
    def forward(self, x):
        return x * torch.sigmoid(x)


def drop_connect(x, p, training):
    if not training:
        return x
    keep = 1.0 - p
    mask = torch.floor(keep + torch.rand([x.shape[0], 1, 1, 1], dtype=x.dtype, device=x.device))
    return x / keep * mask


class MBConvBlock(nn.Module):
    def __init__(self, ba: BlockArgs, gp: GlobalParams, image_size):
        super().__init__()
        self._block_args = ba
        mom, eps = gp.bn_momentum, gp.bn_eps
        mid = ba.inp * ba.expand
        if ba.expand != 1:
            self._expand_conv = StaticSameConv2d(ba.inp, mid, 1, bias=False, image_size=image_size)
            self._bn0 = nn.BatchNorm2d(mid, momentum=mom, eps=eps)
        s = ba.stride if isinstance(ba.stride, int) else ba.stride[0]
        self._depthwise_conv = StaticSameConv2d(mid, mid, ba.kernel, stride=s, groups=mid,
                                                bias=False, image_size=image_size)
        self._bn1 = nn.BatchNorm2d(mid, momentum=mom, eps=eps)
        sq = max(1, int(ba.inp * ba.se_ratio))
        self._se_reduce = StaticSameConv2d(mid, sq, 1, image_size=1)
        self._se_expand = StaticSameConv2d(sq, mid, 1, image_size=1)
        self._project_conv = StaticSameConv2d(mid, ba.out, 1, bias=False,
                                              image_size=int(math.ceil(image_size / s)))
        self._bn2 = nn.BatchNorm2d(ba.out, momentum=mom, eps=eps)
        self._swish = Swish()

    def forward(self, inputs, drop_connect_rate=None):
        ba = self._block_args
        x = inputs
        if ba.expand != 1:
            x = self._swish(self._bn0(self._expand_conv(x)))
        x = self._swish(self._bn1(self._depthwise_conv(x)))
        g = F.adaptive_avg_pool2d(x, 1)
        g = self._se_expand(self._swish(self._se_reduce(g)))
        x = torch.sigmoid(g) * x
        x = self._bn2(self._project_conv(x))
        # list-valued stride of a group's first block never equals 1 (see module docstring)
        if ba.id_skip and ba.stride == 1 and ba.inp == ba.out:
            if drop_connect_rate:
                x = drop_connect(x, drop_connect_rate, self.training)
            x = x + inputs
        return x


class EfficientNet(nn.Module):
    def __init__(self, name="efficientnet-b4", num_classes=1000, drop_connect_rate=0.2):
        super().__init__()
        ver = name.split("-")[1]
        p = {"b4": _B4, "b0": _B0}[ver]
        gp = GlobalParams(p["width"], p["depth"], p["res"], p["dropout"], drop_connect_rate, 0.01, 1e-3)
        self._global_params = gp
        size = gp.image_size
        stem = round_filters(32, gp.width)
        self._conv_stem = StaticSameConv2d(3, stem, 3, stride=2, bias=False, image_size=size)
        self._bn0 = nn.BatchNorm2d(stem, momentum=gp.bn_momentum, eps=gp.bn_eps)
        size = int(math.ceil(size / 2))
        blocks = []
        for r, k, s, e, i, o in _BLOCKS:
            ba = BlockArgs(round_repeats(r, gp.depth), k, [s], e, round_filters(i, gp.width),
                           round_filters(o, gp.width), 0.25, True)
            blocks.append(MBConvBlock(ba, gp, size))
            size = int(math.ceil(size / s))
            rep = ba._replace(inp=ba.out, stride=1)
            for _ in range(ba.repeats - 1):
                blocks.append(MBConvBlock(rep, gp, size))
        self._blocks = nn.ModuleList(blocks)
        last = round_filters(320, gp.width)
        head = round_filters(1280, gp.width)
        self._conv_head = StaticSameConv2d(last, head, 1, bias=False, image_size=size)
        self._bn1 = nn.BatchNorm2d(head, momentum=gp.bn_momentum, eps=gp.bn_eps)
        self._avg_pooling = nn.AdaptiveAvgPool2d(1)
        self._dropout = nn.Dropout(gp.dropout_rate)
        self._fc = nn.Linear(head, num_classes)
        self._swish = Swish()

    @classmethod
    def from_name(cls, name, **kw):
        return cls(name, **kw)

    @classmethod
    def from_pretrained(cls, name, **kw):
        # The real call downloads ImageNet weights; offline, build with local init.
        return cls(name)


# ----------------------------------------------------------------------------------------
# ResNet-18 (torchvision 0.14.1 semantics)
# ----------------------------------------------------------------------------------------

class BasicBlock(nn.Module):
    expansion = 1

    def __init__(self, cin, cout, stride=1, downsample=None):
        super().__init__()
        self.conv1 = nn.Conv2d(cin, cout, 3, stride, 1, bias=False)
        self.bn1 = nn.BatchNorm2d(cout)
        self.relu = nn.ReLU(inplace=True)
        self.conv2 = nn.Conv2d(cout, cout, 3, 1, 1, bias=False)
        self.bn2 = nn.BatchNorm2d(cout)
        self.downsample = downsample
        self.stride = stride

    def forward(self, x):
        y = self.relu(self.bn1(self.conv1(x)))
        y = self.bn2(self.conv2(y))
        idt = x if self.downsample is None else self.downsample(x)
        return self.relu(y + idt)


class ResNet(nn.Module):
    def __init__(self, layers=(2, 2, 2, 2), num_classes=1000, zero_init_residual=False):
        super().__init__()
        self.inplanes = 64
        self.conv1 = nn.Conv2d(3, 64, 7, 2, 3, bias=False)
        self.bn1 = nn.BatchNorm2d(64)
        self.relu = nn.ReLU(inplace=True)
        self.maxpool = nn.MaxPool2d(3, 2, 1)
        self.layer1 = self._make(64, layers[0])
        self.layer2 = self._make(128, layers[1], 2)
        self.layer3 = self._make(256, layers[2], 2)
        self.layer4 = self._make(512, layers[3], 2)
        self.avgpool = nn.AdaptiveAvgPool2d(1)
        self.fc = nn.Linear(512, num_classes)
        for m in self.modules():
            if isinstance(m, nn.Conv2d):
                nn.init.kaiming_normal_(m.weight, mode="fan_out", nonlinearity="relu")
            elif isinstance(m, nn.BatchNorm2d):
                nn.init.constant_(m.weight, 1)
                nn.init.constant_(m.bias, 0)
        if zero_init_residual:
            for m in self.modules():
                if isinstance(m, BasicBlock):
                    nn.init.constant_(m.bn2.weight, 0)

    def _make(self, planes, blocks, stride=1):
        down = None
        if stride != 1 or self.inplanes != planes:
            down = nn.Sequential(nn.Conv2d(self.inplanes, planes, 1, stride, bias=False),
                                 nn.BatchNorm2d(planes))
        mods = [BasicBlock(self.inplanes, planes, stride, down)]
        self.inplanes = planes
        mods += [BasicBlock(planes, planes) for _ in range(1, blocks)]
        return nn.Sequential(*mods)


def resnet18(pretrained=False, progress=True, **kw):
    assert not pretrained, "offline restatement: pretrained weights unavailable"
    return ResNet((2, 2, 2, 2), **kw)
