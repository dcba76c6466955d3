"""Weighted BEV segmentation CE — same class and semantics as reference loss/seg_loss.py."""
from torch import nn

from e2ep_amd import losses


class SegmentationLoss(nn.Module):
    def __init__(self, class_weights):
        super().__init__()
        self.ignore_index = 255
        self.class_weights = class_weights
        self._dev_weights = {}

    def forward(self, pred, target):
        if target.shape[-3] != 1:
            raise ValueError("segmentation label must be index label with channel dim = 1")
        key = str(pred.device)
        w = self._dev_weights.get(key)
        if w is None:  # one H2D copy, then reused (keeps the step free of host copies)
            w = self._dev_weights[key] = self.class_weights.to(pred.device, pred.dtype)
        return losses.seg_weighted_ce(pred, target, w, self.ignore_index)
