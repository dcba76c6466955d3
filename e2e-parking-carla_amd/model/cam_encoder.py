"""Camera encoder: EfficientNet-b4 trunk (blocks 0-21) + DeepLab feature/depth heads.

Mirrors reference model/cam_encoder.py:8-111 (module names and keys); the depth head output
is returned as logits, as in the reference (softmax happens in BevModel)."""
import math

from torch import nn

from e2ep_amd import nn_ops, streams
from model.convolutions import DeepLabHead, UpsamplingConcat
from model.efficientnet import EfficientNetTrunk


class CamEncoder(nn.Module):
    _REDUCTION = {"b4": [0, 24, 32, 56, 160, 448], "b0": [0, 16, 24, 40, 112, 320]}

    def __init__(self, cfg, D):
        super().__init__()
        self.D, self.C = D, cfg.bev_encoder_in_channel
        self.use_depth_distribution = cfg.use_depth_distribution
        self.downsample = cfg.bev_down_sample
        self.version = cfg.backbone.split("-")[1]
        if self.version not in self._REDUCTION:
            raise NotImplementedError(cfg.backbone)
        det = getattr(cfg, "deterministic", False)
        keep = {"b4": 22, "b0": 11}[self.version]
        self.backbone = EfficientNetTrunk(self.version, keep, 0.0 if det else 0.2)
        red = self._REDUCTION[self.version]
        self.index = int(math.log2(self.downsample))
        i = self.index
        p = 0.0 if det else 0.5
        if self.use_depth_distribution:
            self.depth_layer_1 = DeepLabHead(red[i + 1], red[i + 1], 64, p)
            self.depth_layer_2 = UpsamplingConcat(red[i + 1] + red[i], self.D)
        self.feature_layer_1 = DeepLabHead(red[i + 1], red[i + 1], 64, p)
        self.feature_layer_2 = UpsamplingConcat(red[i + 1] + red[i], self.C)

    def get_features_depth(self, x):
        ends = self.backbone(x)
        deep, skip = ends[self.index], ends[self.index - 1]
        depth = None
        if self.use_depth_distribution:
            # both heads read deep and skip: two handles each, gradients summed by one e2ep
            # launch (nn_ops.fork2); the depth head runs on a side stream next to the feature
            # head (e2ep_amd.streams, branch "cam": two chains of 16x16 / 32x32 launches)
            deep, deep_d = nn_ops.fork2(deep)
            skip, skip_d = nn_ops.fork2(skip)
            with streams.branch("cam", x.device, (deep_d, skip_d), self.training) as br:
                depth = self.depth_layer_2(self.depth_layer_1(deep_d), skip_d)
        feature = self.feature_layer_2(self.feature_layer_1(deep), skip)
        if self.use_depth_distribution:
            depth = br.join(depth)
        return feature, depth

    def forward(self, x):
        return self.get_features_depth(x)
