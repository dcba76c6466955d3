"""Camera-head conv blocks with the reference's module/key layout
(reference model/convolutions.py:183-282: UpsamplingConcat, ASPPConv, ASPPPooling, ASPP,
DeepLabHead — the only reachable classes of that file).  Forwards run on e2ep_amd ops."""
import torch
from torch import nn

from e2ep_amd import nn_ops, ops


def _conv_bn(cin, cout, k, pad=0, dil=1):
    return [nn.Conv2d(cin, cout, k, padding=pad, dilation=dil, bias=False), nn.BatchNorm2d(cout),
            nn.ReLU()]


def _run_conv_bn_relu(seq, x, first=0):
    conv, bn = seq[first], seq[first + 1]
    return ops.bn_act(ops.conv2d(x, conv.weight, None, conv.stride, conv.padding, conv.dilation,
                                 bn_stats=bn.training), bn, "relu")


class ASPPConv(nn.Sequential):
    def __init__(self, cin, cout, dilation):
        super().__init__(*_conv_bn(cin, cout, 3, dilation, dilation))

    def forward(self, x):
        return _run_conv_bn_relu(self, x)


class ASPPPooling(nn.Sequential):
    def __init__(self, cin, cout):
        super().__init__(nn.AdaptiveAvgPool2d(1), *_conv_bn(cin, cout, 1))

    def forward(self, x):
        g = _run_conv_bn_relu(self, ops.global_avg_pool(x), first=1)
        return ops.resize(g, x.shape[-2:])


class ASPP(nn.Module):
    def __init__(self, cin, rates, cout=256, p_drop=0.5):
        super().__init__()
        mods = [nn.Sequential(*_conv_bn(cin, cout, 1))]
        mods += [ASPPConv(cin, cout, r) for r in rates]
        mods.append(ASPPPooling(cin, cout))
        self.convs = nn.ModuleList(mods)
        self.project = nn.Sequential(*_conv_bn(len(mods) * cout, cout, 1), nn.Dropout(p_drop))

    def forward(self, x):
        # x feeds five branches: it is threaded through the four conv branches as each conv's
        # skip alias (e2ep_amd.conv.conv2d skip=True), so its gradient is summed inside the
        # branch convs' data-gradient epilogues instead of by four autograd adds
        branches = []
        for m in self.convs[:-1]:
            conv, bn = m[0], m[1]
            c, x = ops.conv2d(x, conv.weight, None, conv.stride, conv.padding, conv.dilation,
                              skip=True, bn_stats=bn.training)
            branches.append(ops.bn_act(c, bn, "relu"))
        branches.append(self.convs[-1](x))
        y = _run_conv_bn_relu(self.project, nn_ops.cat_channels(branches))
        # Dropout(0.5) after the project BN-ReLU (reference model/convolutions.py:264): y >= 0,
        # so dropout(y) = dropout(relu(y)) runs on the fused ReLU-dropout kernel, one launch
        # each way (its backward's relu mask only drops entries whose BN-ReLU gradient is 0)
        p = self.project[3].p if self.training else 0.0
        if p > 0.0:
            y = nn_ops.relu_dropout(y, p)
        return y


class DeepLabHead(nn.Sequential):
    def __init__(self, cin, cout, hidden_channel=256, p_drop=0.5):
        super().__init__(ASPP(cin, (12, 24, 36), hidden_channel, p_drop),
                         nn.Conv2d(hidden_channel, hidden_channel, 3, padding=1, bias=False),
                         nn.BatchNorm2d(hidden_channel), nn.ReLU(), nn.Conv2d(hidden_channel, cout, 1))

    def forward(self, x):
        y = self[0](x)
        y = ops.bn_act(ops.conv2d(y, self[1].weight, None, 1, 1, bn_stats=self[2].training),
                       self[2], "relu")
        return ops.conv2d(y, self[4].weight, self[4].bias)


class UpsamplingConcat(nn.Module):
    def __init__(self, cin, cout, scale_factor=2):
        super().__init__()
        self.upsample = nn.Upsample(scale_factor=scale_factor, mode="bilinear", align_corners=False)
        self.conv = nn.Sequential(*_conv_bn(cin, cout, 3, 1), *_conv_bn(cout, cout, 3, 1))

    def forward(self, x_to_upsample, x):
        y = nn_ops.cat_channels([x, ops.upsample2x(x_to_upsample)])
        y = _run_conv_bn_relu(self.conv, y, 0)
        return _run_conv_bn_relu(self.conv, y, 3)
