"""Convolution autograd op over the e2ep implicit-GEMM kernels (csrc/conv.hip).

conv2d(x, w, b, stride, padding(l,r,t,b), dilation, act) -> y, with backward through
e2ep_conv_dgrad / e2ep_conv_wgrad / e2ep_bias_grad.  groups must be 1 (depthwise convs use
e2ep_amd.dwconv).  The im2col k-tables are built once per geometry on the device and cached.
"""
import torch

from . import _lib, timing

_TABLES = {}


def _table(dims, dgrad, device):
    key = (tuple(dims), dgrad, str(device))
    t = _TABLES.get(key)
    if t is None:
        n = (dims[4] if dgrad else dims[1]) * dims[5] * dims[6]
        t = torch.empty(n * 4, dtype=torch.int32, device=device)
        d = _lib.dims(dims)
        _lib.call("e2ep_conv_table", d, int(dgrad), _lib.ptr(t), _lib.stream())
        _TABLES[key] = t
    return t


def _splits(dims):
    N, Cin, H, W, Cout, R, S, P, Q = dims[:9]
    Kg = Cin * R * S
    base = -(-Kg // 128) * -(-Cout // 64)
    pix = N * P * Q
    want = max(1, -(-512 // base))
    return int(max(1, min(want, pix // 256, 64)))


class _Conv2d(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, w, b, dims, act):
        x = x.contiguous()
        w = w.contiguous()
        N, Cin, H, W, Cout, R, S, P, Q = dims[:9]
        y = torch.empty(N, Cout, P, Q, dtype=torch.float32, device=x.device)
        d = _lib.dims(dims)
        with timing.region("conv_fwd"):
            _lib.call("e2ep_conv_fwd", _lib.ptr(x), _lib.ptr(w), _lib.ptr(b),
                      _lib.ptr(_table(dims, 0, x.device)), d, act, _lib.ptr(y), _lib.stream())
        ctx.dims, ctx.act, ctx.has_bias = dims, act, b is not None
        ctx.save_for_backward(x, w, y if act else None)
        return y

    @staticmethod
    def backward(ctx, gy):
        x, w, y = ctx.saved_tensors
        dims = ctx.dims
        N, Cin, H, W, Cout, R, S, P, Q = dims[:9]
        gy = gy.contiguous()
        if ctx.act == 1:
            gy = torch.where(y > 0, gy, torch.zeros((), device=gy.device))
        d = _lib.dims(dims)
        s = _lib.stream()
        dx = dw = db = None
        if ctx.needs_input_grad[0]:
            dx = torch.empty_like(x)
            with timing.region("conv_dgrad"):
                _lib.call("e2ep_conv_dgrad", _lib.ptr(gy), _lib.ptr(w),
                          _lib.ptr(_table(dims, 1, x.device)), d, _lib.ptr(dx), s)
        if ctx.needs_input_grad[1]:
            splits = _splits(dims)
            ws = torch.empty(splits * Cout * Cin * R * S, dtype=torch.float32, device=x.device)
            dw = torch.empty_like(w)
            with timing.region("conv_wgrad"):
                _lib.call("e2ep_conv_wgrad", _lib.ptr(gy), _lib.ptr(x),
                          _lib.ptr(_table(dims, 0, x.device)), d, splits, _lib.ptr(ws),
                          _lib.ptr(dw), 0, s)
        if ctx.has_bias and ctx.needs_input_grad[2]:
            db = torch.empty(Cout, dtype=torch.float32, device=x.device)
            _lib.call("e2ep_bias_grad", _lib.ptr(gy), N, Cout, P * Q, _lib.ptr(db), s)
        return dx, dw, db, None, None


def conv2d(x, w, b=None, stride=(1, 1), pad=(0, 0, 0, 0), dilation=(1, 1), act=0):
    """pad = (left, right, top, bottom); act 0 none, 1 relu (fused epilogue)."""
    if not x.is_cuda:
        raise _lib.E2EPError("e2ep conv2d runs on a HIP device only")
    N, Cin, H, W = x.shape
    Cout, cin_w, R, S = w.shape
    if cin_w != Cin:
        raise _lib.E2EPError(f"e2ep conv2d: groups must be 1 (w {tuple(w.shape)}, x {tuple(x.shape)})")
    sh, sw = stride
    dh, dw = dilation
    l, r, t, btm = pad
    P = (H + t + btm - dh * (R - 1) - 1) // sh + 1
    Q = (W + l + r - dw * (S - 1) - 1) // sw + 1
    dims = (N, Cin, H, W, Cout, R, S, P, Q, sh, sw, t, l, dh, dw)
    return _Conv2d.apply(x, w, b, dims, act)
