"""Training module with the reference's LightningModule API (trainer/pl_trainer.py:14-121).

`ParkingTrainingModule(cfg)` exposes training_step / validation_step / configure_optimizers
and the `parking_model` attribute (so checkpoints keep the `parking_model.` key prefix that
agent/parking_agent.py:261 strips).  PyTorch-Lightning is not part of this image: when it is
importable the class derives from `pl.LightningModule` and plugs into the reference's
pl_train.py unchanged; otherwise it is a plain nn.Module driven by e2ep_amd.train.
"""
import torch
from torch import nn

from loss.control_loss import ControlLoss, ControlValLoss
from loss.depth_loss import DepthLoss
from loss.seg_loss import SegmentationLoss
from e2ep_amd import nn_ops
from model.parking_model import ParkingModel

try:  # pragma: no cover - PL absent in this image
    import pytorch_lightning as pl
    _Base = pl.LightningModule
    HAVE_PL = True
except Exception:  # noqa: BLE001
    _Base = nn.Module
    HAVE_PL = False


def setup_callbacks(cfg):
    """Checkpoint (top-3 on val_loss + last), progress, summary and LR-monitor callbacks when
    PyTorch-Lightning is available (trainer/pl_trainer.py:14-33); [] otherwise."""
    if not HAVE_PL:
        return []
    from pytorch_lightning.callbacks import (LearningRateMonitor, ModelCheckpoint, ModelSummary,
                                             TQDMProgressBar)
    return [ModelCheckpoint(dirpath=cfg.checkpoint_dir, monitor="val_loss", save_top_k=3, mode="min",
                            filename="E2EParking-{epoch:02d}-{val_loss:.2f}", save_last=True),
            TQDMProgressBar(), ModelSummary(max_depth=2), LearningRateMonitor(logging_interval="epoch")]


class ParkingTrainingModule(_Base):
    def __init__(self, cfg):
        super().__init__()
        if HAVE_PL:
            self.save_hyperparameters()
        self.cfg = cfg
        self.control_loss_func = ControlLoss(cfg)
        self.control_val_loss_func = ControlValLoss(cfg)
        self.segmentation_loss_func = SegmentationLoss(
            class_weights=torch.Tensor(cfg.seg_vehicle_weights))
        self.depth_loss_func = DepthLoss(cfg)
        self.parking_model = ParkingModel(cfg)
        self.logged = {}

    if not HAVE_PL:
        def log_dict(self, d, **_):
            self.logged = {k: v.detach() for k, v in d.items()}

    def compute_losses(self, batch, noise=None):
        pred_control, pred_segmentation, pred_depth = self.parking_model(batch, noise)
        out = {
            "control_loss": self.control_loss_func(pred_control, batch),
            "segmentation_loss": self.segmentation_loss_func(pred_segmentation.unsqueeze(1),
                                                             batch["segmentation"]),
            "depth_loss": self.depth_loss_func(pred_depth, batch["depth"]),
        }
        a, b, c = out["control_loss"], out["segmentation_loss"], out["depth_loss"]
        # (a + b) + c as the reference sums them; one e2ep launch on the device
        out["train_loss"] = nn_ops.sum3(a, b, c) if a.is_cuda else a + b + c
        return out, (pred_control, pred_segmentation, pred_depth)

    def training_step(self, batch, batch_idx=0, noise=None):
        loss_dict, _ = self.compute_losses(batch, noise)
        self.log_dict(loss_dict)
        return loss_dict["train_loss"]

    def validation_step(self, batch, batch_idx=0, noise=None):
        pred_control, pred_segmentation, pred_depth = self.parking_model(batch, noise)
        acc_steer, reverse = self.control_val_loss_func(pred_control, batch)
        d = {"acc_steer_val_loss": acc_steer, "reverse_val_loss": reverse,
             "segmentation_val_loss": self.segmentation_loss_func(pred_segmentation.unsqueeze(1),
                                                                  batch["segmentation"]),
             "depth_val_loss": self.depth_loss_func(pred_depth, batch["depth"])}
        d["val_loss"] = sum(d.values())
        self.log_dict(d)
        return d["val_loss"]

    def configure_optimizers(self):
        """Adam(lr, weight_decay) + CosineAnnealingLR(T_max=epochs), as the reference
        (trainer/pl_trainer.py:116-121).  On a HIP device the optimizer is the fused flat Adam
        (same update; the schedule reaches its captured launches through a device LR scalar);
        parameters that never receive a gradient (bev_encoder.layer4, reference
        model/bev_encoder.py:21) are not stepped by either optimizer."""
        params = [p for p in self.parameters() if p.requires_grad]
        if params and params[0].is_cuda:
            from e2ep_amd.optim import FlatAdam
            opt = FlatAdam(params, lr=self.cfg.learning_rate, weight_decay=self.cfg.weight_decay)
        else:
            opt = torch.optim.Adam(params, lr=self.cfg.learning_rate,
                                   weight_decay=self.cfg.weight_decay)
        sched = torch.optim.lr_scheduler.CosineAnnealingLR(optimizer=opt, T_max=self.cfg.epochs)
        return {"optimizer": opt, "lr_scheduler": sched}
