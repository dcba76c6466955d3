"""PyTorch-Lightning-format checkpoints without PyTorch-Lightning.

The reference trains under PL 1.5 (trainer/pl_trainer.py:17-22 ModelCheckpoint, :39
save_hyperparameters) and its agent loads `ckpt['state_dict']`, stripping the
`parking_model.` prefix (agent/parking_agent.py:257-262).  PL is not part of this image, so
this module writes and reads the same on-disk layout directly:

    {"epoch", "global_step", "pytorch-lightning_version", "state_dict" (parking_model.* keys),
     "callbacks" {state_key: state}, "optimizer_states" [torch.optim.Adam format],
     "lr_schedulers" [CosineAnnealingLR state], "hparams_name": "kwargs",
     "hyper_parameters" {"cfg": tool.config.Configuration}}

`hyper_parameters["cfg"]` pickles as `tool.config.Configuration`, the reference's own module
path, so either code base unpickles it into its own Configuration class.  Reading never
executes arbitrary pickled code: torch.load(weights_only=True) with only
tool.config.Configuration (and torch.device) allow-listed; a checkpoint holding any other
Python object is rejected with the loader's error.
"""
import collections

import torch

PL_VERSION = "1.5.0"
PREFIX = "parking_model."


def _safe_globals():
    from tool.config import Configuration
    return [Configuration, torch.device]


def checkpoint_dict(module, optimizer=None, lr_scheduler=None, epoch=0, global_step=0,
                    callbacks=None):
    """The dict PL 1.5's ModelCheckpoint would save for ParkingTrainingModule `module`."""
    state = collections.OrderedDict((k, v.detach().cpu()) for k, v in module.state_dict().items())
    opt_states = []
    if optimizer is not None:
        sd = optimizer.state_dict()
        sd = {"state": {i: {k: (v.detach().cpu() if torch.is_tensor(v) else v)
                            for k, v in s.items()} for i, s in sd["state"].items()},
              "param_groups": sd["param_groups"]}
        opt_states.append(sd)
    return {"epoch": int(epoch), "global_step": int(global_step),
            "pytorch-lightning_version": PL_VERSION, "state_dict": state,
            "callbacks": dict(callbacks or {}), "optimizer_states": opt_states,
            "lr_schedulers": [lr_scheduler.state_dict()] if lr_scheduler is not None else [],
            "hparams_name": "kwargs", "hyper_parameters": {"cfg": module.cfg}}


def save_checkpoint(path, module, optimizer=None, lr_scheduler=None, epoch=0, global_step=0,
                    callbacks=None):
    torch.save(checkpoint_dict(module, optimizer, lr_scheduler, epoch, global_step, callbacks), path)


def load_checkpoint(path, map_location="cpu"):
    """Read a PL-format checkpoint (ours or the reference's) with the restricted unpickler."""
    with torch.serialization.safe_globals(_safe_globals()):
        return torch.load(path, map_location=map_location, weights_only=True)


def model_state_dict(ckpt):
    """agent/parking_agent.py:261: ckpt['state_dict'] with the `parking_model.` prefix removed."""
    return collections.OrderedDict((k.replace(PREFIX, ""), v) for k, v in ckpt["state_dict"].items())


def load_parking_model(path, cfg=None, device=None):
    """ParkingAgent.load_model (agent/parking_agent.py:257-264): build ParkingModel(cfg) (cfg
    from the checkpoint's hyper-parameters when not given), load the weights strictly, move
    to `device` and switch to eval mode."""
    from model.parking_model import ParkingModel
    ckpt = load_checkpoint(path)
    if cfg is None:
        cfg = ckpt["hyper_parameters"]["cfg"]
    model = ParkingModel(cfg)
    model.load_state_dict(model_state_dict(ckpt))
    if device is not None:
        model = model.to(device)
    return model.eval()


def restore_training(ckpt, module, optimizer=None, lr_scheduler=None):
    """Load weights, optimizer and LR-scheduler state from a checkpoint dict into a
    ParkingTrainingModule and its optimizers (resuming a run)."""
    module.load_state_dict(ckpt["state_dict"])
    if optimizer is not None and ckpt.get("optimizer_states"):
        optimizer.load_state_dict(ckpt["optimizer_states"][0])
    if lr_scheduler is not None and ckpt.get("lr_schedulers"):
        lr_scheduler.load_state_dict(ckpt["lr_schedulers"][0])
    return ckpt.get("epoch", 0), ckpt.get("global_step", 0)
