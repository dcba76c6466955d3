"""Weighted BEV segmentation CE — same class and semantics as reference loss/seg_loss.py."""
from torch import nn

from e2ep_amd import losses


class SegmentationLoss(nn.Module):
    def __init__(self, class_weights):
        super().__init__()
        self.ignore_index = 255
        self.class_weights = class_weights

    def forward(self, pred, target):
        if target.shape[-3] != 1:
            raise ValueError("segmentation label must be index label with channel dim = 1")
        return losses.seg_weighted_ce(pred, target, self.class_weights, self.ignore_index)
