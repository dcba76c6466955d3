"""BEV encoder: bilinear 200->256, conv7x7/2 65->64, BN, ReLU, maxpool, ResNet-18 layer1-3.

Mirrors reference model/bev_encoder.py:8-36 with torchvision-0.14.1 key names
(conv1, bn1, layer1..layer4; BasicBlock conv1/bn1/conv2/bn2/downsample.{0,1}).  layer4 is
constructed (its weights are part of the checkpoint contract) but, as in the reference,
never run, so it receives no gradient and is excluded from the gradient all-reduce."""
import torch
from torch import nn

from e2ep_amd import bev_stem, ops


class BasicBlock(nn.Module):
    expansion = 1

    def __init__(self, cin, cout, stride=1):
        super().__init__()
        self.conv1 = nn.Conv2d(cin, cout, 3, stride, 1, bias=False)
        self.bn1 = nn.BatchNorm2d(cout)
        self.relu = nn.ReLU(inplace=True)
        self.conv2 = nn.Conv2d(cout, cout, 3, 1, 1, bias=False)
        self.bn2 = nn.BatchNorm2d(cout)
        self.downsample = None
        if stride != 1 or cin != cout:
            self.downsample = nn.Sequential(nn.Conv2d(cin, cout, 1, stride, bias=False),
                                            nn.BatchNorm2d(cout))
        self.stride = stride

    def forward(self, x):
        # identity skip, or the downsample conv's input: x is conv1's skip alias either way, so
        # its second gradient joins conv1's data gradient in the epilogue (no autograd add)
        # bn_stats: each BN's batch statistics from its conv's epilogue where it takes them
        c1, x = ops.conv2d(x, self.conv1.weight, None, self.stride, 1, skip=True,
                           bn_stats=self.bn1.training)
        y = ops.bn_act(c1, self.bn1, "relu")
        if self.downsample is not None:
            ds = self.downsample[1]
            x = ops.bn_act(ops.conv2d(x, self.downsample[0].weight, None, self.stride, 0,
                                      bn_stats=ds.training), ds, None)
        # relu(bn2(conv2(y)) + identity) as one fused BN/residual/activation kernel
        return ops.bn_act(ops.conv2d(y, self.conv2.weight, None, 1, 1, bn_stats=self.bn2.training),
                          self.bn2, "relu", res=x)


def _layer(cin, cout, stride):
    return nn.Sequential(BasicBlock(cin, cout, stride), BasicBlock(cout, cout, 1))


class BevEncoder(nn.Module):
    def __init__(self, in_channel):
        super().__init__()
        self.conv1 = nn.Conv2d(in_channel + 1, 64, kernel_size=7, stride=2, padding=3, bias=False)
        self.bn1 = nn.BatchNorm2d(64)
        self.relu = nn.ReLU(inplace=True)
        self.max_pool = nn.MaxPool2d(3, 2, 1)
        self.layer1 = _layer(64, 64, 1)
        self.layer2 = _layer(64, 128, 2)
        self.layer3 = _layer(128, 256, 2)
        self.layer4 = _layer(256, 512, 2)
        for m in self.modules():  # torchvision init, zero_init_residual=True
            if isinstance(m, nn.Conv2d):
                nn.init.kaiming_normal_(m.weight, mode="fan_out", nonlinearity="relu")
            elif isinstance(m, nn.BatchNorm2d):
                nn.init.ones_(m.weight)
                nn.init.zeros_(m.bias)
        for m in self.modules():
            if isinstance(m, BasicBlock):
                nn.init.zeros_(m.bn2.weight)
        self.conv1.reset_parameters()  # the reference's own conv1 keeps PyTorch's default init

    def forward(self, x):
        """x: (B, 65, 200, 200) — 64 pooled BEV channels + the target plane."""
        return self.forward_split(x[:, :-1], x[:, -1:])

    def forward_split(self, bev, target):
        """Same as forward(cat(bev, target)) without materialising the concatenation; the
        target plane is a constant (no gradient), as in the reference."""
        x = bev_stem.bev_stem(bev, target, self.conv1.weight, (256, 256))
        x = ops.bn_act(x, self.bn1, "relu")
        x = ops.max_pool3s2(x)
        x = self.layer3(self.layer2(self.layer1(x)))
        return torch.flatten(x, 2)
