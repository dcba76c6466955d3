"""BEV segmentation head: tokens -> 16x16 map -> top-down 1x1 convs with x2 upsampling ->
resize to 200x200 -> 3x3 conv + BN + ReLU -> 1x1 conv to the class logits.

Mirrors reference model/segmentation_head.py:10-47 (keys: c5_conv, up_conv5/4/3,
segmentation_head.{0,1,3})."""
import math

import torch
from torch import nn

from e2ep_amd import nn_ops, ops


class SegmentationHead(nn.Module):
    def __init__(self, cfg):
        super().__init__()
        self.cfg = cfg
        self.in_channel = cfg.bev_encoder_out_channel
        self.out_channel = cfg.bev_encoder_in_channel
        self.seg_classes = cfg.seg_classes
        c = self.out_channel
        self.relu = nn.ReLU(inplace=True)
        self.up_sample = nn.Upsample(scale_factor=2, mode="bilinear", align_corners=False)
        self.c5_conv = nn.Conv2d(self.in_channel, c, (1, 1))
        self.up_conv5 = nn.Conv2d(c, c, (1, 1))
        self.up_conv4 = nn.Conv2d(c, c, (1, 1))
        self.up_conv3 = nn.Conv2d(c, c, (1, 1))
        self.segmentation_head = nn.Sequential(
            nn.Conv2d(c, c, kernel_size=3, padding=1, bias=False), nn.BatchNorm2d(c),
            nn.ReLU(inplace=True), nn.Conv2d(c, self.seg_classes, kernel_size=1, padding=0))

    def top_down(self, x):
        x = ops.conv2d(x, self.c5_conv.weight, self.c5_conv.bias, act="relu")
        for conv in (self.up_conv5, self.up_conv4, self.up_conv3):
            x = ops.conv2d(ops.upsample2x(x), conv.weight, conv.bias, act="relu")
        return ops.resize(x, (200, 200))

    def forward(self, fuse_feature):
        t = nn_ops.transpose12(fuse_feature)  # (B, S, C) tokens -> (B, C, S), one launch
        b, c, s = t.shape
        x = self.top_down(t.reshape(b, c, int(math.sqrt(s)), -1))
        head = self.segmentation_head
        x = ops.bn_act(ops.conv2d(x, head[0].weight, None, 1, 1, bn_stats=head[1].training),
                       head[1], "relu")
        return ops.conv2d(x, head[3].weight, head[3].bias)
