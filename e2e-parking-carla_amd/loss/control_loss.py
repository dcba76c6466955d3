"""Control-token losses — same classes and semantics as reference loss/control_loss.py."""
import torch
from torch import nn

from e2ep_amd import losses


class ControlLoss(nn.Module):
    def __init__(self, cfg):
        super().__init__()
        self.cfg = cfg
        self.pad_idx = cfg.token_nums - 1

    def forward(self, pred, data):
        return losses.control_ce(pred, data["gt_control"], self.pad_idx)


class ControlValLoss(nn.Module):
    """Validation metrics (reference loss/control_loss.py:22-75): SmoothL1 on detokenised
    acc/steer and a 2-way CE on the reverse token mass.  Detokenisation is vectorised (the
    reference loops in Python over acc tokens); values are identical."""

    def __init__(self, cfg):
        super().__init__()
        self.cfg = cfg
        self.pad_idx = cfg.token_nums - 1
        self.valid_token = cfg.token_nums - 4
        self.half_token = float(self.valid_token / 2)
        self.ce_loss = nn.CrossEntropyLoss(ignore_index=self.pad_idx)
        self.l1_loss = nn.SmoothL1Loss()

    def forward(self, pred, data):
        ctrl = pred[:, :-2, :]
        acc_tok = torch.softmax(ctrl[:, 0::3, :], dim=-1).argmax(dim=-1).reshape(-1).float()
        ht = self.half_token
        acc = torch.where(acc_tok > ht, acc_tok / ht - 1, -(acc_tok / ht - 1))
        acc_loss = self.l1_loss(acc, data["gt_acc"].reshape(-1).to(pred.device))
        steer_tok = torch.softmax(ctrl[:, 1::3, :], dim=-1).argmax(dim=-1).reshape(-1)
        steer = steer_tok / ht - 1
        steer_loss = self.l1_loss(steer, data["gt_steer"].reshape(-1).to(pred.device))
        rev = torch.softmax(ctrl[:, 2::3, :], dim=-1)
        p_no = rev[:, :, :101].sum(-1).reshape(-1)
        p_yes = rev[:, :, 101:].sum(-1).reshape(-1)
        rev_loss = self.ce_loss(torch.stack((p_no, p_yes), dim=0).T,
                                data["gt_reverse"].reshape(-1).to(pred.device))
        return acc_loss + steer_loss, rev_loss
