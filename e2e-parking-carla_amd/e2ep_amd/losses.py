"""Loss arithmetic of the hot path (reference loss/*.py).  Kept in one place so the fused HIP
loss kernels can replace each function without touching the nn.Module wrappers."""
import torch
import torch.nn.functional as F


def control_ce(pred, gt_control, pad_idx):
    """loss/control_loss.py:15-19: CE over (B*14, vocab) vs gt[:, 1:], PAD ignored."""
    return F.cross_entropy(pred.reshape(-1, pred.shape[-1]),
                           gt_control[:, 1:].reshape(-1).to(pred.device), ignore_index=pad_idx)


def seg_weighted_ce(pred, target, weights, ignore_index=255):
    """loss/seg_loss.py:12-26: per-pixel weighted CE, then a plain mean over pixels."""
    b, s, c, h, w = pred.shape
    l = F.cross_entropy(pred.view(b * s, c, h, w), target.view(b * s, h, w).to(pred.device),
                        reduction="none", ignore_index=ignore_index,
                        weight=weights.to(device=pred.device, dtype=pred.dtype))
    return l.mean()


def depth_onehot(gt, d_bound, down):
    """loss/depth_loss.py:31-48: min non-zero depth per down x down cell -> one-hot bin."""
    B, N, H, W = gt.shape
    D = int((d_bound[1] - d_bound[0]) / d_bound[2])
    g = gt.view(B * N, H // down, down, W // down, down, 1).permute(0, 1, 3, 5, 2, 4).contiguous()
    g = g.view(-1, down * down)
    g = torch.where(g == 0.0, 1e5 * torch.ones_like(g), g).min(-1).values
    g = (g - (d_bound[0] - d_bound[2])) / d_bound[2]
    g = torch.where((g < D + 1) & (g >= 0.0), g, torch.zeros_like(g))
    return F.one_hot(g.long(), num_classes=D + 1).view(-1, D + 1)[:, 1:].float()


def depth_bce(prob, gt, d_bound, down):
    """loss/depth_loss.py:18-28: BCE on foreground cells, summed / max(1, #fg).

    The reference selects the foreground rows with a boolean index (a data-dependent shape,
    i.e. a device->host sync); here every row is evaluated and the background rows are
    multiplied by 0, which gives the same sum without a sync (graph-capturable).  BCE keeps
    PyTorch's log clamp at -100."""
    lab = depth_onehot(gt.to(prob.device), d_bound, down)
    D = lab.shape[1]
    p = prob.permute(0, 2, 3, 1).reshape(-1, D)
    fg = (lab.max(dim=1).values > 0.0).to(prob.dtype)
    ll = lab * torch.clamp(torch.log(p), min=-100.0) + (1 - lab) * torch.clamp(torch.log1p(-p), min=-100.0)
    return -(ll.sum(dim=1) * fg).sum() / fg.sum().clamp(min=1.0)
