"""The three training losses (reference loss/*.py) as autograd ops over the fused HIP loss
kernels (csrc/loss.hip): two launches forward (rows/blocks -> one fixed-order final sum),
one backward, no host synchronisation, no PyTorch arithmetic.  The nn.Module wrappers in
loss/ keep the reference's classes and signatures."""
import torch

from . import _lib


def _dev(*ts):
    for t in ts:
        if t is not None and not t.is_cuda:
            raise _lib.E2EPError("e2ep losses run on a HIP device only; got a CPU tensor")


def _i64(t, device):
    return t.to(device=device, dtype=torch.int64, non_blocking=True).contiguous()


def _ws(nbytes, device):
    return torch.empty(max(int(nbytes), 16), dtype=torch.uint8, device=device)


class _ControlCE(torch.autograd.Function):
    @staticmethod
    def forward(ctx, pred, gt, pad):
        pred = pred.contiguous()
        B, T, V = pred.shape
        f32 = dict(dtype=torch.float32, device=pred.device)
        loss, lse, count = torch.empty((), **f32), torch.empty(B * T, **f32), torch.empty(1, **f32)
        ws = _ws(_lib.load().e2ep_control_ce_workspace(B * T), pred.device)
        _lib.call("e2ep_control_ce_fwd", _lib.ptr(pred), _lib.ptr(gt), B, T, gt.shape[1], 1, V, pad,
                  _lib.ptr(loss), _lib.ptr(lse), _lib.ptr(count), _lib.ptr(ws), _lib.stream())
        ctx.save_for_backward(pred, gt, lse, count)
        ctx.pad = pad
        return loss

    @staticmethod
    def backward(ctx, g):
        pred, gt, lse, count = ctx.saved_tensors
        B, T, V = pred.shape
        d = torch.empty_like(pred)
        _lib.call("e2ep_control_ce_bwd", _lib.ptr(pred), _lib.ptr(gt), _lib.ptr(lse), _lib.ptr(count),
                  _lib.ptr(g.contiguous()), B, T, gt.shape[1], 1, V, ctx.pad, _lib.ptr(d), _lib.stream())
        return d, None, None


def control_ce(pred, gt_control, pad_idx):
    """loss/control_loss.py:15-19: CE over (B*T, vocab) logits vs gt[:, 1:], PAD ignored.
    pred (B, T, vocab) fp32, gt_control (B, T+1) token ids."""
    _dev(pred)
    gt = _i64(gt_control, pred.device)
    if pred.dim() != 3 or gt.shape[1] != pred.shape[1] + 1 or gt.shape[0] != pred.shape[0]:
        raise _lib.E2EPError(f"control_ce: pred {tuple(pred.shape)} vs gt_control {tuple(gt.shape)}")
    return _ControlCE.apply(pred, gt, int(pad_idx))


class _SegCE(torch.autograd.Function):
    @staticmethod
    def forward(ctx, pred, target, weights, ignore):
        pred = pred.contiguous()
        n, C = pred.shape[0], pred.shape[1]
        HW = pred[0, 0].numel()
        loss = torch.empty((), dtype=torch.float32, device=pred.device)
        ws = _ws(_lib.load().e2ep_seg_ce_workspace(n, HW), pred.device)
        _lib.call("e2ep_seg_ce_fwd", _lib.ptr(pred), _lib.ptr(target), _lib.ptr(weights), n, C, HW,
                  ignore, _lib.ptr(loss), _lib.ptr(ws), _lib.stream())
        ctx.save_for_backward(pred, target, weights)
        ctx.ignore = ignore
        return loss

    @staticmethod
    def backward(ctx, g):
        pred, target, weights = ctx.saved_tensors
        n, C = pred.shape[0], pred.shape[1]
        HW = pred[0, 0].numel()
        d = torch.empty_like(pred)
        _lib.call("e2ep_seg_ce_bwd", _lib.ptr(pred), _lib.ptr(target), _lib.ptr(weights),
                  _lib.ptr(g.contiguous()), n, C, HW, ctx.ignore, _lib.ptr(d), _lib.stream())
        return d, None, None, None


def seg_weighted_ce(pred, target, weights, ignore_index=255):
    """loss/seg_loss.py:12-26: per-pixel weighted CE, then a plain mean over pixels.
    pred (b, s, C, H, W) logits, target (b, s, H, W) class ids, weights (C,)."""
    _dev(pred)
    b, s, c, h, w = pred.shape
    tg = _i64(target, pred.device).view(b * s, h * w)
    wt = weights.to(device=pred.device, dtype=torch.float32).contiguous()
    return _SegCE.apply(pred.reshape(b * s, c, h, w), tg, wt, int(ignore_index))


def depth_onehot(gt, d_bound, down):
    """loss/depth_loss.py:31-48 (get_down_sampled_gt_depth): min non-zero depth per down x down
    cell -> one-hot bin labels (B*N*h*w, D).  The loss itself derives the labels inside its
    kernel; this is the reference's public helper."""
    B, N, H, W = gt.shape
    D = int((d_bound[1] - d_bound[0]) / d_bound[2])
    g = gt.view(B * N, H // down, down, W // down, down, 1).permute(0, 1, 3, 5, 2, 4).contiguous()
    g = g.view(-1, down * down)
    g = torch.where(g == 0.0, 1e5 * torch.ones_like(g), g).min(-1).values
    g = (g - (d_bound[0] - d_bound[2])) / d_bound[2]
    g = torch.where((g < D + 1) & (g >= 0.0), g, torch.zeros_like(g))
    return torch.nn.functional.one_hot(g.long(), num_classes=D + 1).view(-1, D + 1)[:, 1:].float()


class _DepthBCE(torch.autograd.Function):
    @staticmethod
    def forward(ctx, prob, gt, down, lo, step):
        prob = prob.contiguous()
        BN, D, h, w = prob.shape
        H, W = gt.shape[-2:]
        dev = prob.device
        loss = torch.empty((), dtype=torch.float32, device=dev)
        den = torch.empty(1, dtype=torch.float32, device=dev)
        cls = torch.empty(BN * h * w, dtype=torch.int32, device=dev)
        ws = _ws(_lib.load().e2ep_depth_bce_workspace(BN, H, W, down), dev)
        fn = "e2ep_depth_bce_fwd_f64" if gt.dtype == torch.float64 else "e2ep_depth_bce_fwd"
        _lib.call(fn, _lib.ptr(prob), _lib.ptr(gt), BN, D, H, W, down, lo, step,
                  _lib.ptr(loss), _lib.ptr(den), _lib.ptr(cls), _lib.ptr(ws), _lib.stream())
        ctx.save_for_backward(prob, cls, den)
        return loss

    @staticmethod
    def backward(ctx, g):
        prob, cls, den = ctx.saved_tensors
        BN, D, h, w = prob.shape
        d = torch.empty_like(prob)
        _lib.call("e2ep_depth_bce_bwd", _lib.ptr(prob), _lib.ptr(cls), _lib.ptr(den),
                  _lib.ptr(g.contiguous()), BN, D, h * w, _lib.ptr(d), _lib.stream())
        return d, None, None, None, None


def depth_bce(prob, gt, d_bound, down):
    """loss/depth_loss.py:18-28: BCE on the foreground cells, summed / max(1, #fg).
    prob (B*N, D, H/down, W/down) probabilities, gt (B, N, H, W) metric depth."""
    _dev(prob)
    B, N, H, W = gt.shape
    D = int((d_bound[1] - d_bound[0]) / d_bound[2])
    if prob.shape != (B * N, D, H // down, W // down):
        raise _lib.E2EPError(f"depth_bce: prob {tuple(prob.shape)} vs gt {tuple(gt.shape)}")
    # float64 depth (what the reference dataset yields) keeps float64 bin arithmetic; any other
    # dtype is promoted/rounded to fp32, as torch computes on a float32 tensor
    dt = torch.float64 if gt.dtype == torch.float64 else torch.float32
    g = gt.to(device=prob.device, dtype=dt, non_blocking=True).contiguous()
    lo = float(d_bound[0] - d_bound[2])  # evaluated in Python double, applied in the gt dtype
    return _DepthBCE.apply(prob, g, int(down), lo, float(d_bound[2]))
