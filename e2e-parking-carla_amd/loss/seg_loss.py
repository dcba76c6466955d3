"""Weighted BEV segmentation CE — same class and semantics as reference loss/seg_loss.py."""
import torch
from torch import nn

from e2ep_amd import losses


class SegmentationLoss(nn.Module):
    def __init__(self, class_weights):
        super().__init__()
        self.ignore_index = 255
        # a non-persistent buffer: Module.to() moves it with the training module (no host copy
        # inside the step, nor inside a capture-only process's graph), and the state dict keeps
        # the reference's keys (the reference holds a plain tensor attribute)
        self.register_buffer("class_weights", torch.as_tensor(class_weights), persistent=False)
        self._dev_weights = {}

    def forward(self, pred, target):
        if target.shape[-3] != 1:
            raise ValueError("segmentation label must be index label with channel dim = 1")
        w = self.class_weights
        if w.device != pred.device or w.dtype != pred.dtype:
            key = (str(pred.device), pred.dtype)
            w = self._dev_weights.get(key)
            if w is None:  # one H2D copy, then reused
                w = self._dev_weights[key] = self.class_weights.to(pred.device, pred.dtype)
        return losses.seg_weighted_ce(pred, target, w, self.ignore_index)
