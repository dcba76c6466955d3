"""BEV-encoder stem as one autograd op: bilinear 200->256 of the 64 pooled BEV channels and
the target-point plane, then conv7x7/2 (65->64) — reference model/bev_encoder.py:24-27.

Forward writes the two resizes straight into one (B, 65, 256, 256) buffer (no torch.cat of
the target channel, reference model/parking_model.py:45).  Backward computes the data
gradient for the 64 feature channels only (the target plane is a constant), resizes it
back to 200x200 with the deterministic gather straight into a channels-last (pillar-major)
tensor — the lift-splat backward reads it without a transpose — and the weight gradient
with the split-K kernel."""
import torch

from . import _lib, conv, timing


class _BevStem(torch.autograd.Function):
    @staticmethod
    def forward(ctx, bev, tgt, w, size):
        B, C, X, Y = bev.shape
        H, W = size
        assert bev.stride(3) == 1 and bev.stride(2) == Y and bev.stride(1) == X * Y
        tgt = tgt.contiguous()
        Cin = C + 1
        x = torch.empty(B, Cin, H, W, dtype=torch.float32, device=bev.device)
        s = _lib.stream()
        sh, sw = X / H, Y / W
        with timing.region("resize_fwd"):
            _lib.call("e2ep_resize_fwd", _lib.ptr(bev), B, C, bev.stride(0), X, Y, H, W, sh, sw,
                      _lib.ptr(x), Cin * H * W, s)
            _lib.call("e2ep_resize_fwd", _lib.ptr(tgt), B, 1, X * Y, X, Y, H, W, sh, sw,
                      _lib.ptr(x[:, C:]), Cin * H * W, s)
        Cout, _, R, S = w.shape
        P, Q = (H + 6 - R) // 2 + 1, (W + 6 - S) // 2 + 1
        dims = (B, Cin, H, W, Cout, R, S, P, Q, 2, 2, 3, 3, 1, 1)
        wt = conv.tap_major(w)
        y = conv.conv_fwd(x, wt, None, dims, 0,
                          torch.empty(B, Cout, P, Q, dtype=torch.float32, device=bev.device), w_layout=1)
        ctx.save_for_backward(x, w, wt)
        ctx.meta = (B, C, X, Y, H, W, sh, sw, dims)
        return y

    @staticmethod
    def backward(ctx, gy):
        x, w, wt = ctx.saved_tensors
        B, C, X, Y, H, W, sh, sw, dims = ctx.meta
        gy = gy.contiguous()
        s = _lib.stream()
        d = _lib.dims(dims)
        dbev = dw = None
        fork = None
        if ctx.needs_input_grad[2]:  # weight gradient on the side stream (conv._Fork)
            dw = torch.empty_like(w)
            ws = torch.empty(_lib.load().e2ep_conv_wgrad_splits(d) * dw.numel(), dtype=torch.float32,
                             device=gy.device)
            fork = conv._Fork(gy.device, on=ctx.needs_input_grad[0],
                              work_us=conv.est_us(conv.conv_flops(dims)))
            with fork:
                conv.conv_wgrad(gy, x, dims, dw, ws)
        if ctx.needs_input_grad[0]:
            dres = conv.conv_dgrad(gy, wt, dims, C,
                                   torch.empty(B, C, H, W, dtype=torch.float32, device=gy.device), w_layout=1)
            # channels-last (pillar-major [B][X*Y][C]): the layout the lift-splat backward
            # gathers rows of, so it needs no transpose of the BEV gradient
            dbev = torch.empty(B, C, X, Y, dtype=torch.float32, device=gy.device,
                               memory_format=torch.channels_last)
            with timing.region("resize_bwd"):
                _lib.call("e2ep_resize_bwd_cl", _lib.ptr(dres), H * W, B, C, X, Y, H, W, sh, sw,
                          _lib.ptr(dbev), s)
        if fork is not None:
            fork.join()
        return dbev, None, dw, None


def bev_stem(bev, tgt, weight, size=(256, 256)):
    """conv7x7/2(resize(cat(bev, tgt)))  with bev (B,C,X,Y) [grad], tgt (B,1,X,Y) [const]."""
    if not bev.is_cuda:
        raise _lib.E2EPError("e2ep bev_stem runs on a HIP device only")
    return _BevStem.apply(bev, tgt.detach(), weight, tuple(size))
