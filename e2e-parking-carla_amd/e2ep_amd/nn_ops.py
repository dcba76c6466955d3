"""Autograd ops over the e2ep BN / resize / depthwise / pooling / SE kernels (csrc/bn.hip,
resize.hip, dwconv.hip, pool.hip).  Each forward enqueues on torch's current HIP stream;
each backward is the matching e2ep gradient kernel (no PyTorch arithmetic)."""
import ctypes
import os

import torch
import torch.nn.functional as F

from . import _lib, conv, rng, timing

ACT = {None: 0, "none": 0, "relu": 1, "swish": 2}


def _dev(*ts):
    for t in ts:
        if t is not None and not t.is_cuda:
            raise _lib.E2EPError("e2ep ops run on a HIP device only; got a CPU tensor")


def _ws(nbytes, device):
    return torch.empty(max(int(nbytes), 16), dtype=torch.uint8, device=device)


# bf16 activation storage (C3, e2ep.h E2EP_IO_*): in a bf16-precision training forward the
# MBConv depthwise output (the squeeze-excitation's input) is stored bf16, and so are the two
# activation gradients on either side of the depthwise conv (the gradient at that output, and
# the depthwise data gradient feeding _bn0's backward); statistics, parameters and their
# gradients stay fp32.  E2EP_BF16_STORE: 0 (default) keeps every activation fp32, 1 stores the
# depthwise output (and the two gradients beside it) bf16, 2 also the squeeze-excitation
# output — the project conv's input — and the gradient at it.  Off by default: level 2 saves
# 0.27 ms of the 18.4 ms C3 step (most of these tensors are presumably served from the 256 MB MALL, not
# HBM) and puts the step's gradient-norm median error above the bf16 AMP comparator's
# (0.0355 vs 0.0318; level 1: 0.0362) — profiles/r05/bf16_store_ab.txt.
_IO_X, _IO_DY, _IO_DX = 1, 2, 4
_BF16_STORE = [int(os.environ.get("E2EP_BF16_STORE", "0"))]


def set_bf16_store(level):
    """Set the bf16 activation storage level of the C3 mode (0 off, 1 depthwise output, 2 also
    the squeeze-excitation output; True = 2); returns the previous level."""
    prev = _BF16_STORE[0]
    _BF16_STORE[0] = int(level) * (2 if level is True else 1)
    return prev


def _store_bf16(train, level=1):
    if not (train and _BF16_STORE[0] >= level):
        return False
    from . import precision
    return precision.get() == "bf16"


def _is_bf16(t):
    return t is not None and t.dtype == torch.bfloat16



# ------------------------------------------------------------------------------------------
# BatchNorm2d + activation (+ residual)
# ------------------------------------------------------------------------------------------
class _BnAct(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, gamma, beta, res, rm, rv, train, momentum, eps, act, dc_rand, dc_keep,
                part=None, tiles=0):
        x = x.contiguous()
        res = res.contiguous() if res is not None else None
        N, C, H, W = x.shape
        y = torch.empty_like(x)
        if part is not None and train:
            # statistics from the producing conv's epilogue (e2ep_conv_fwd_stats): finalize the
            # partials, then the elementwise pass with the folded affine
            st = torch.empty(4, C, dtype=torch.float32, device=x.device)  # mean, invstd, scale, shift
            mean, invstd = st[0], st[1]
            with timing.region(timing.name("bn_fwd", x.shape, "_BnAct")):
                fws = _ws(_lib.load().e2ep_bn_finalize_part_workspace(C, tiles), x.device)
                _lib.call("e2ep_bn_finalize_part", _lib.ptr(part), tiles, _lib.ptr(gamma),
                          _lib.ptr(beta), _lib.ptr(rm), _lib.ptr(rv), N, C, H, W, float(momentum),
                          float(eps), _lib.ptr(st[0]), _lib.ptr(st[1]), _lib.ptr(st[2]),
                          _lib.ptr(st[3]), _lib.ptr(fws), _lib.nbytes(fws), _lib.stream())
                _lib.call("e2ep_bn_apply", _lib.ptr(x), _lib.ptr(st[2]), _lib.ptr(st[3]),
                          _lib.ptr(res), _lib.ptr(dc_rand), float(dc_keep), N, C, H, W, act,
                          _lib.ptr(y), _lib.stream())
            ctx.save_for_backward(x, gamma, beta, res, mean, invstd, dc_rand)
            ctx.train, ctx.act, ctx.dc_keep = train, act, dc_keep
            return y
        mean = torch.empty(C, dtype=torch.float32, device=x.device)
        invstd = torch.empty_like(mean)
        ws = _ws(_lib.load().e2ep_bn_workspace(N, C, H, W), x.device)
        with timing.region(timing.name("bn_fwd", x.shape, "_BnAct")):
            _lib.call("e2ep_bn_fwd", _lib.ptr(x), _lib.ptr(gamma), _lib.ptr(beta), _lib.ptr(res),
                      _lib.ptr(dc_rand), float(dc_keep), _lib.ptr(rm), _lib.ptr(rv), N, C, H, W,
                      int(train), float(momentum), float(eps), act, _lib.ptr(mean),
                      _lib.ptr(invstd), _lib.ptr(y), _lib.ptr(ws), _lib.nbytes(ws), _lib.stream())
        ctx.save_for_backward(x, gamma, beta, res, mean, invstd, dc_rand)
        ctx.train, ctx.act, ctx.dc_keep = train, act, dc_keep
        return y

    @staticmethod
    def backward(ctx, dy):
        x, gamma, beta, res, mean, invstd, dc_rand = ctx.saved_tensors
        dy = dy.contiguous()
        N, C, H, W = x.shape
        nig = ctx.needs_input_grad
        dx = torch.empty_like(x) if nig[0] else None
        dg = torch.empty_like(gamma) if (gamma is not None and nig[1]) else None
        db = torch.empty_like(beta) if (beta is not None and nig[2]) else None
        # no activation: the residual's gradient is dy itself (y = dc(bn(x)) + res) — hand dy
        # over instead of writing a copy
        dres_is_dy = res is not None and nig[3] and ctx.act == 0
        dres = torch.empty_like(x) if (res is not None and nig[3] and not dres_is_dy) else None
        ws = _ws(_lib.load().e2ep_bn_workspace(N, C, H, W), x.device)
        with timing.region(timing.name("bn_bwd", x.shape, "_BnAct")):
            _lib.call("e2ep_bn_bwd", _lib.ptr(x), _lib.ptr(dy), _lib.ptr(mean), _lib.ptr(invstd),
                      _lib.ptr(gamma), _lib.ptr(beta), _lib.ptr(res), _lib.ptr(dc_rand),
                      float(ctx.dc_keep), None, None, N, C, H, W, int(ctx.train), ctx.act, _lib.ptr(dx),
                      _lib.ptr(dg), _lib.ptr(db), _lib.ptr(dres), _lib.ptr(ws), _lib.nbytes(ws), _lib.stream(),
                      0)
        if dres_is_dy:
            dres = dy
        return dx, dg, db, dres, None, None, None, None, None, None, None, None, None, None


class BnCounters:
    """num_batches_tracked bookkeeping for a whole model in one launch per forward.

    BatchNorm2d increments its counter on every training forward.  The first training forward
    of a model runs with per-layer increments while it records which BN layers ran (the
    BEV encoder's layer4 never does, reference model/bev_encoder.py:21,23-36); later forwards
    suppress the per-layer increments and add 1 to all recorded counters with one
    torch._foreach_add_ — same counter values, ~100 fewer launches per step."""

    def __init__(self):
        self.recorded = None  # BN modules, in call order
        self._log = None
        self.batched = False

    def __enter__(self):
        if self.recorded is None:
            self._log = []
        else:
            ctrs = [bn.num_batches_tracked for bn in self.recorded]
            key = tuple(c.data_ptr() for c in ctrs)
            if getattr(self, "_table_key", None) == key:
                # one e2ep launch over the device table of the counters' addresses
                _lib.call("e2ep_add_i64_multi", _lib.ptr(self._table), len(ctrs), 1, _lib.stream())
            else:
                torch._foreach_add_(ctrs, 1)
            self.batched = True
        _COUNTERS.append(self)
        return self

    def __exit__(self, *exc):
        _COUNTERS.pop()
        if self.recorded is None and self._log is not None and not exc[0]:
            self.recorded = self._log
            ctrs = [bn.num_batches_tracked for bn in self.recorded]
            # the device table of counter addresses for later forwards (the buffers live as
            # long as the modules), built here, outside any graph capture: the first forward
            # runs eagerly
            if (ctrs and all(c.is_cuda and c.dtype == torch.int64 for c in ctrs)
                    and not torch.cuda.is_current_stream_capturing()):
                self._table = torch.tensor([c.data_ptr() for c in ctrs], dtype=torch.int64,
                                           device=ctrs[0].device)
                self._table_key = tuple(c.data_ptr() for c in ctrs)
        self._log = None
        self.batched = False
        return False

    def note(self, bn):
        if self.batched:
            return
        bn.num_batches_tracked.add_(1)
        if self._log is not None:
            self._log.append(bn)


_COUNTERS = []  # stack of active BnCounters (innermost last)


class EvalBnBatch:
    """Eval statistics (mean, invstd, folded scale / shift) of every BatchNorm whose
    normalisation an inference forward hands to a fused consumer (the depthwise conv's and the
    squeeze-excitation's input transforms) in ONE launch at scope entry (e2ep_bn_eval_multi)
    instead of one e2ep_bn_stats launch per layer (42 of C5 predict's launches).

    The first forward inside the scope records the BN modules in call order (each computing its
    own statistics); later forwards compute every recorded layer's statistics into one
    persistent buffer (stable addresses, so a captured predict graph replays the launch) and
    hand out views.  Active only without autograd (torch.no_grad, the predict / agent path): a
    view is rewritten by the next forward, so it must not be saved for a backward.  A layer that
    was not recorded, or whose buffers moved, computes its own statistics."""

    def __init__(self):
        self.recorded = None
        self._log = None
        self._views = {}
        self._key = None
        self._table = None
        self._buf = None
        self.active = False

    @staticmethod
    def _key_of(bns):
        return [(b.running_mean.data_ptr(), b.running_var.data_ptr(),
                 b.weight.data_ptr() if b.weight is not None else 0,
                 b.bias.data_ptr() if b.bias is not None else 0, b.num_features, float(b.eps))
                for b in bns]

    def _build(self, bns):
        import struct
        dev = bns[0].running_mean.device
        self._buf = torch.empty(4 * sum(b.num_features for b in bns), dtype=torch.float32, device=dev)
        rows, views, off = [], [], 0
        for b in bns:
            C = b.num_features
            v = self._buf[off:off + 4 * C].view(4, C)
            eps_bits = struct.unpack("<i", struct.pack("<f", float(b.eps)))[0]
            rows.append([b.running_mean.data_ptr(), b.running_var.data_ptr(),
                         b.weight.data_ptr() if b.weight is not None else 0,
                         b.bias.data_ptr() if b.bias is not None else 0, v.data_ptr(), C, eps_bits])
            views.append(v)
            off += 4 * C
        self._table = torch.tensor(rows, dtype=torch.int64).to(dev)
        self._key = self._key_of(bns)
        self._vlist = views

    def __enter__(self):
        self.active = not torch.is_grad_enabled()
        if self.active:
            bns = self.recorded
            if bns is None:
                self._log = []
            elif self._key_of(bns) != self._key:
                self.recorded, self._log = None, []  # buffers moved: record again
            else:
                _lib.call("e2ep_bn_eval_multi", _lib.ptr(self._table), len(bns), _lib.stream())
                self._views = {id(b): v for b, v in zip(bns, self._vlist)}
        _EVAL_BN.append(self)
        return self

    def __exit__(self, *exc):
        _EVAL_BN.pop()
        if (self.active and self.recorded is None and self._log and not exc[0]
                and not torch.cuda.is_current_stream_capturing()):  # host->device table copy
            log = [b for b in self._log if b.track_running_stats and b.running_mean.is_cuda]
            if 0 < len(log) <= 4096:
                self.recorded = log
                self._build(log)
        self._log = None
        self._views = {}
        self.active = False
        return False

    def lookup(self, bn):
        if not self.active:
            return None
        v = self._views.get(id(bn))
        if v is None and self._log is not None and all(bn is not o for o in self._log):
            self._log.append(bn)
        return v


_EVAL_BN = []  # active EvalBnBatch scopes (innermost last)


def _eval_bn_stats(bn):
    """This eval BN's (4, C) statistics from the active EvalBnBatch launch, or None."""
    if not _EVAL_BN or not bn.track_running_stats or torch.is_grad_enabled():
        return None
    return _EVAL_BN[-1].lookup(bn)


def _bn_train_and_count(bn):
    """BatchNorm2d.forward's mode choice and num_batches_tracked increment."""
    if bn.training and bn.track_running_stats:
        if _COUNTERS:
            _COUNTERS[-1].note(bn)
        else:
            bn.num_batches_tracked.add_(1)
    return bn.training or not bn.track_running_stats


def batch_norm_act(x, bn, act=None, res=None, dc_rand=None, dc_keep=1.0):
    """BatchNorm2d module `bn` (its train/eval mode, momentum, eps, running buffers) applied
    to x, then optional drop-connect (dc_rand: per-sample uniform draws, training only), an
    optional residual, then the activation."""
    _dev(x, res, dc_rand)
    train = _bn_train_and_count(bn)
    rm = bn.running_mean if bn.track_running_stats else None
    rv = bn.running_var if bn.track_running_stats else None
    mom = bn.momentum if bn.momentum is not None else 0.1
    if dc_rand is not None:
        dc_rand = dc_rand.contiguous()
    pp = conv.bn_partials(x) if train else None
    return _BnAct.apply(x, bn.weight, bn.bias, res, rm, rv, train, mom, bn.eps, ACT[act],
                        dc_rand, dc_keep, *(pp or (None, 0)))


class _Act(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, act):
        x = x.contiguous()
        y = torch.empty_like(x)
        _lib.call("e2ep_act_fwd", _lib.ptr(x), x.numel(), act, _lib.ptr(y), _lib.stream())
        ctx.save_for_backward(x)
        ctx.act = act
        return y

    @staticmethod
    def backward(ctx, dy):
        (x,) = ctx.saved_tensors
        dy = dy.contiguous()
        dx = torch.empty_like(x)
        _lib.call("e2ep_act_bwd", _lib.ptr(x), _lib.ptr(dy), x.numel(), ctx.act, _lib.ptr(dx),
                  _lib.stream())
        return dx, None


def activation(x, act):
    _dev(x)
    return _Act.apply(x, ACT[act])


# ------------------------------------------------------------------------------------------
# bilinear resize (align_corners=False)
# ------------------------------------------------------------------------------------------
class _Resize(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, Ho, Wo, sh, sw):
        x = x.contiguous()
        N, C, Hi, Wi = x.shape
        y = torch.empty(N, C, Ho, Wo, dtype=torch.float32, device=x.device)
        with timing.region(timing.name("resize_fwd", x.shape, "_Resize")):
            _lib.call("e2ep_resize_fwd", _lib.ptr(x), N, C, C * Hi * Wi, Hi, Wi, Ho, Wo, sh, sw,
                      _lib.ptr(y), C * Ho * Wo, _lib.stream())
        ctx.meta = (N, C, Hi, Wi, Ho, Wo, sh, sw)
        return y

    @staticmethod
    def backward(ctx, g):
        N, C, Hi, Wi, Ho, Wo, sh, sw = ctx.meta
        g = g.contiguous()
        gx = torch.empty(N, C, Hi, Wi, dtype=torch.float32, device=g.device)
        ws = _ws(N * C * Ho * Wi * 4, g.device)
        with timing.region(timing.name("resize_bwd", g.shape, "_Resize")):
            _lib.call("e2ep_resize_bwd", _lib.ptr(g), Ho * Wo, N * C, Hi, Wi, Ho, Wo, sh, sw,
                      _lib.ptr(gx), 0, _lib.ptr(ws), _lib.stream())
        return gx, None, None, None, None


def resize(x, size=None, scale_factor=None):
    """F.interpolate(x, size | scale_factor, mode='bilinear', align_corners=False)."""
    _dev(x)
    Hi, Wi = x.shape[-2:]
    if scale_factor is not None:
        Ho, Wo = int(Hi * scale_factor), int(Wi * scale_factor)
        sh = sw = 1.0 / float(scale_factor)
    else:
        Ho, Wo = size
        sh, sw = Hi / Ho, Wi / Wo
    return _Resize.apply(x, int(Ho), int(Wo), float(sh), float(sw))


# ------------------------------------------------------------------------------------------
# depthwise conv
# Both gradients of a stride-1 depthwise layer in one launch (e2ep_dwconv_bwd, k_dw_bwd_pair)
# where e2ep_dwconv_bwd_pair_ok: no fork / join.  E2EP_DW_PAIR=0 keeps the forked two-launch
# backward (A/B).
_DW_PAIR = [os.environ.get("E2EP_DW_PAIR", "1") != "0"]


def set_dw_pair(on):
    """Enable / disable the one-launch depthwise backward (returns the previous setting)."""
    prev = _DW_PAIR[0]
    _DW_PAIR[0] = bool(on)
    return prev


def _dw_pairable(d):
    return _DW_PAIR[0] and _lib.load().e2ep_dwconv_bwd_pair_ok(d) == 1


# ------------------------------------------------------------------------------------------
class _DwConv(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, w, dims, ystats=None):
        x = x.contiguous()
        w = w.contiguous()
        N, C, H, W, K, P, Q = dims[:7]
        y = torch.empty(N, C, P, Q, dtype=torch.float32, device=x.device)
        d = _lib.dims(dims)
        with timing.region(timing.name("dwconv_fwd", x.shape, "_DwConv")):
            _lib.call("e2ep_dwconv_fwd_stats", _lib.ptr(x), _lib.ptr(w), d, None, None, 0,
                      _lib.ptr(y), _lib.ptr(ystats), _lib.nbytes(ystats), _lib.stream(), 0)
        ctx.save_for_backward(x, w)
        ctx.dims = dims
        return y

    @staticmethod
    def backward(ctx, gy):
        x, w = ctx.saved_tensors
        gy = gy.contiguous()
        d = _lib.dims(ctx.dims)
        s = _lib.stream()
        dx = dw = None
        if ctx.needs_input_grad[0] and ctx.needs_input_grad[1] and _dw_pairable(d):
            dx, dw = torch.empty_like(x), torch.empty_like(w)
            ws = _ws(_lib.load().e2ep_dwconv_wgrad_workspace(d), x.device)
            with timing.region(timing.name("dwconv_bwd", gy.shape, "_DwConv")):
                _lib.call("e2ep_dwconv_bwd", _lib.ptr(gy), _lib.ptr(x), _lib.ptr(w), d, None, None, 0,
                          _lib.ptr(dx), _lib.ptr(ws), _lib.nbytes(ws), _lib.ptr(dw), s, 0)
            return dx, dw, None, None
        fork = None
        if ctx.needs_input_grad[1]:  # weight gradient on the side stream (conv._Fork)
            dw = torch.empty_like(w)
            ws = _ws(_lib.load().e2ep_dwconv_wgrad_workspace(d), x.device)
            fork = conv._Fork(x.device, on=ctx.needs_input_grad[0],
                              work_us=conv.est_us(nbytes=4.0 * (x.numel() + gy.numel())))
            with fork, timing.region(timing.name("dwconv_wgrad", gy.shape, "_DwConv")):
                _lib.call("e2ep_dwconv_wgrad", _lib.ptr(gy), _lib.ptr(x), d, None, None, 0,
                          _lib.ptr(ws), _lib.nbytes(ws), _lib.ptr(dw), _lib.stream(), 0)
        if ctx.needs_input_grad[0]:
            dx = torch.empty_like(x)
            with timing.region(timing.name("dwconv_dgrad", gy.shape, "_DwConv")):
                _lib.call("e2ep_dwconv_dgrad", _lib.ptr(gy), _lib.ptr(w), d, _lib.ptr(dx), s, 0)
        if fork is not None:
            fork.join()
        return dx, dw, None, None


class _BnActDwConv(torch.autograd.Function):
    """depthwise_conv(act(bn(x))) with the BN + activation applied while the depthwise
    kernel stages its input: the normalised tensor is never stored (MBConv's
    _bn0 -> swish -> _depthwise_conv, reference model/cam_encoder.py:70-72 via
    efficientnet-pytorch MBConvBlock.forward).  Same arithmetic as batch_norm_act followed by
    depthwise_conv2d."""

    @staticmethod
    def forward(ctx, x, gamma, beta, rm, rv, train, momentum, eps, act, w, dims, part=None, tiles=0,
                ystats=None, pre=None):
        x = x.contiguous()
        w = w.contiguous()
        N, C, H, W, K, P, Q = dims[:7]
        f32 = dict(dtype=torch.float32, device=x.device)
        stats = pre if pre is not None else torch.empty(4, C, **f32)  # mean, invstd, scale, shift
        s = _lib.stream()
        with timing.region(timing.name("bn_fwd", x.shape, "_BnActDwConv")):
            if pre is not None:  # eval statistics of the forward's EvalBnBatch launch
                pass
            elif part is not None and train:  # partials from the expand conv's epilogue
                fws = _ws(_lib.load().e2ep_bn_finalize_part_workspace(C, tiles), x.device)
                _lib.call("e2ep_bn_finalize_part", _lib.ptr(part), tiles, _lib.ptr(gamma),
                          _lib.ptr(beta), _lib.ptr(rm), _lib.ptr(rv), N, C, H, W, float(momentum),
                          float(eps), _lib.ptr(stats[0]), _lib.ptr(stats[1]), _lib.ptr(stats[2]),
                          _lib.ptr(stats[3]), _lib.ptr(fws), _lib.nbytes(fws), s)
            else:
                ws = _ws(_lib.load().e2ep_bn_workspace(N, C, H, W), x.device)
                _lib.call("e2ep_bn_stats", _lib.ptr(x), _lib.ptr(gamma), _lib.ptr(beta), _lib.ptr(rm),
                          _lib.ptr(rv), N, C, H, W, int(train), float(momentum), float(eps),
                          _lib.ptr(stats[0]), _lib.ptr(stats[1]), _lib.ptr(stats[2]),
                          _lib.ptr(stats[3]), _lib.ptr(ws), _lib.nbytes(ws), s, 0)
        # bf16 storage of the depthwise output (C3 training, _store_bf16)
        d = _lib.dims(dims)
        # every kernel on either side of this layer must take the bf16 masks, or the layer
        # keeps fp32 storage (e2ep_dwconv_bf16_ok: forward, data / weight gradients, the BNs)
        hb = _store_bf16(train) and _lib.call_raw("e2ep_dwconv_bf16_ok", d) == 1
        y = torch.empty(N, C, P, Q, dtype=torch.bfloat16 if hb else torch.float32, device=x.device)
        with timing.region(timing.name("dwconv_fwd", x.shape, "_BnActDwConv")):
            _lib.call("e2ep_dwconv_fwd_stats", _lib.ptr(x), _lib.ptr(w), d, _lib.ptr(stats[2]),
                      _lib.ptr(stats[3]), act, _lib.ptr(y), _lib.ptr(ystats), _lib.nbytes(ystats), s,
                      _IO_DX if hb else 0)
        ctx.save_for_backward(x, gamma, beta, w, stats)
        ctx.dims, ctx.train, ctx.act = dims, train, act
        return y

    @staticmethod
    def backward(ctx, gy):
        x, gamma, beta, w, stats = ctx.saved_tensors
        gy = gy.contiguous()
        N, C, H, W = x.shape
        d = _lib.dims(ctx.dims)
        s = _lib.stream()
        nig = ctx.needs_input_grad
        dw = dx = dg = db = None
        fork = None
        want_t = nig[0] or nig[1] or nig[2]
        paired = nig[9] and want_t and _dw_pairable(d)
        # bf16 storage: the incoming gradient (at the stored bf16 output) is bf16, and so is the
        # data gradient handed to the BN backward
        hb = _is_bf16(gy)
        tdt = torch.bfloat16 if hb else torch.float32
        if paired:  # both gradients in one launch
            dw = torch.empty_like(w)
            dt = torch.empty(x.shape, dtype=tdt, device=x.device)  # gradient at the activation output
            wsw = _ws(_lib.load().e2ep_dwconv_wgrad_workspace(d), x.device)
            with timing.region(timing.name("dwconv_bwd", gy.shape, "_BnActDwConv")):
                _lib.call("e2ep_dwconv_bwd", _lib.ptr(gy), _lib.ptr(x), _lib.ptr(w), d,
                          _lib.ptr(stats[2]), _lib.ptr(stats[3]), ctx.act, _lib.ptr(dt),
                          _lib.ptr(wsw), _lib.nbytes(wsw), _lib.ptr(dw), s,
                          (_IO_DY | _IO_DX) if hb else 0)
        elif nig[9]:  # weight gradient on the side stream (conv._Fork)
            dw = torch.empty_like(w)
            wsw = _ws(_lib.load().e2ep_dwconv_wgrad_workspace(d), x.device)
            fork = conv._Fork(x.device, on=want_t,
                              work_us=conv.est_us(nbytes=4.0 * (x.numel() + gy.numel())))
            with fork, timing.region(timing.name("dwconv_wgrad", gy.shape, "_BnActDwConv")):
                _lib.call("e2ep_dwconv_wgrad", _lib.ptr(gy), _lib.ptr(x), d, _lib.ptr(stats[2]),
                          _lib.ptr(stats[3]), ctx.act, _lib.ptr(wsw), _lib.nbytes(wsw), _lib.ptr(dw), _lib.stream(),
                          _IO_DY if hb else 0)
        if want_t:
            if not paired:
                dt = torch.empty(x.shape, dtype=tdt, device=x.device)  # gradient at the activation output
                with timing.region(timing.name("dwconv_dgrad", gy.shape, "_BnActDwConv")):
                    _lib.call("e2ep_dwconv_dgrad", _lib.ptr(gy), _lib.ptr(w), d, _lib.ptr(dt), s,
                              (_IO_DY | _IO_DX) if hb else 0)
            dx = torch.empty_like(x) if nig[0] else None
            dg = torch.empty_like(gamma) if (gamma is not None and nig[1]) else None
            db = torch.empty_like(beta) if (beta is not None and nig[2]) else None
            ws = _ws(_lib.load().e2ep_bn_workspace(N, C, H, W), x.device)
            with timing.region(timing.name("bn_bwd", x.shape, "_BnActDwConv")):
                _lib.call("e2ep_bn_bwd", _lib.ptr(x), _lib.ptr(dt), _lib.ptr(stats[0]),
                          _lib.ptr(stats[1]), _lib.ptr(gamma), _lib.ptr(beta), None, None, 1.0,
                          None, None, N, C, H, W, int(ctx.train), ctx.act, _lib.ptr(dx), _lib.ptr(dg),
                          _lib.ptr(db), None, _lib.ptr(ws), _lib.nbytes(ws), s, _IO_DY if hb else 0)
        if fork is not None:
            fork.join()
        return dx, dg, db, None, None, None, None, None, None, dw, None, None, None, None, None


def depthwise_conv2d(x, w, stride, pad, bn_stats=False):
    """pad = (left, right, top, bottom); w [C, 1, K, K].  bn_stats: see
    bn_act_depthwise_conv2d."""
    _dev(x)
    N, C, H, W = x.shape
    K = w.shape[-1]
    l, r, t, b = pad
    P = (H + t + b - K) // stride + 1
    Q = (W + l + r - K) // stride + 1
    dims = (N, C, H, W, K, P, Q, stride, t, l)
    ys, tiles = _dw_stats_buffer(dims, x.device, bn_stats)
    y = _DwConv.apply(x, w, dims, ys)
    if ys is not None:
        y._e2ep_bn_part = (ys, tiles)
    return y


def _dw_stats_buffer(dims, device, want):
    """(fp64 partials buffer, tiles) for the depthwise forward's BatchNorm statistics
    (e2ep_dwconv_fwd_stats), or (None, 0) when not wanted or the kernel takes none."""
    lib = _lib.load()
    if not want or not conv._BN_STATS[0] or not lib.e2ep_bn_fwd_split(dims[0], dims[1], dims[5], dims[6]):
        return None, 0
    tiles = lib.e2ep_dwconv_fwd_stats_tiles(_lib.dims(dims))
    if tiles <= 0:
        return None, 0
    return torch.empty(dims[1] * tiles * 2, dtype=torch.float64, device=device), tiles


def bn_act_depthwise_conv2d(x, bn, act, w, stride, pad, bn_stats=False):
    """depthwise_conv2d(batch_norm_act(x, bn, act), w, stride, pad) as one fused op.
    bn_stats: a training BatchNorm reads the output next (its partial sums come from the
    depthwise kernel, attached as for conv.conv2d(bn_stats=True))."""
    _dev(x)
    train = _bn_train_and_count(bn)
    rm = bn.running_mean if bn.track_running_stats else None
    rv = bn.running_var if bn.track_running_stats else None
    mom = bn.momentum if bn.momentum is not None else 0.1
    N, C, H, W = x.shape
    K = w.shape[-1]
    l, r, t, b = pad
    P = (H + t + b - K) // stride + 1
    Q = (W + l + r - K) // stride + 1
    pp = conv.bn_partials(x) if train else None
    dims = (N, C, H, W, K, P, Q, stride, t, l)
    ys, tiles = _dw_stats_buffer(dims, x.device, bn_stats)
    y = _BnActDwConv.apply(x, bn.weight, bn.bias, rm, rv, train, mom, bn.eps, ACT[act], w, dims,
                           *(pp or (None, 0)), ys, None if train else _eval_bn_stats(bn))
    if ys is not None:
        y._e2ep_bn_part = (ys, tiles)
    return y


# ------------------------------------------------------------------------------------------
# pooling / SE gate
# ------------------------------------------------------------------------------------------
class _MaxPool(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x):
        x = x.contiguous()
        N, C, H, W = x.shape
        P, Q = (H - 1) // 2 + 1, (W - 1) // 2 + 1
        y = torch.empty(N, C, P, Q, dtype=torch.float32, device=x.device)
        arg = torch.empty(N, C, P, Q, dtype=torch.int8, device=x.device)
        _lib.call("e2ep_maxpool3s2_fwd", _lib.ptr(x), N * C, H, W, _lib.ptr(y), _lib.ptr(arg),
                  _lib.stream())
        ctx.save_for_backward(arg)
        ctx.shape = x.shape
        return y

    @staticmethod
    def backward(ctx, gy):
        (arg,) = ctx.saved_tensors
        N, C, H, W = ctx.shape
        dx = torch.empty(N, C, H, W, dtype=torch.float32, device=gy.device)
        _lib.call("e2ep_maxpool3s2_bwd", _lib.ptr(gy.contiguous()), _lib.ptr(arg), N * C, H, W,
                  _lib.ptr(dx), _lib.stream())
        return dx


def max_pool3s2(x):
    _dev(x)
    return _MaxPool.apply(x)


class _AvgPool(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x):
        x = x.contiguous()
        N, C, H, W = x.shape
        y = torch.empty(N, C, 1, 1, dtype=torch.float32, device=x.device)
        _lib.call("e2ep_avgpool_fwd", _lib.ptr(x), N * C, H * W, _lib.ptr(y), _lib.stream())
        ctx.shape = x.shape
        return y

    @staticmethod
    def backward(ctx, gy):
        N, C, H, W = ctx.shape
        dx = torch.empty(N, C, H, W, dtype=torch.float32, device=gy.device)
        _lib.call("e2ep_avgpool_bwd", _lib.ptr(gy.contiguous()), N * C, H * W, _lib.ptr(dx),
                  _lib.stream())
        return dx


def global_avg_pool(x):
    _dev(x)
    return _AvgPool.apply(x)


class _SeGate(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, a):
        x = x.contiguous()
        a = a.contiguous()
        N, C, H, W = x.shape
        y = torch.empty_like(x)
        with timing.region(timing.name("se_gate_fwd", x.shape, "_SeGate")):
            _lib.call("e2ep_se_gate_fwd", _lib.ptr(x), _lib.ptr(a), N * C, H * W, _lib.ptr(y),
                      _lib.stream())
        ctx.save_for_backward(x, a)
        return y

    @staticmethod
    def backward(ctx, dy):
        x, a = ctx.saved_tensors
        N, C, H, W = x.shape
        dx = torch.empty_like(x)
        da = torch.empty_like(a)
        with timing.region(timing.name("se_gate_bwd", x.shape, "_SeGate")):
            _lib.call("e2ep_se_gate_bwd", _lib.ptr(x), _lib.ptr(a), _lib.ptr(dy.contiguous()), N * C,
                      H * W, _lib.ptr(dx), _lib.ptr(da), _lib.stream())
        return dx, da


def se_gate(x, a):
    """x * sigmoid(a), a [N, C, 1, 1]."""
    _dev(x, a)
    return _SeGate.apply(x, a)


# ------------------------------------------------------------------------------------------
# squeeze-and-excitation (fused)
# ------------------------------------------------------------------------------------------
class _SqueezeExcite(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, w1, b1, w2, b2):
        x = x.contiguous()
        N, C, H, W = x.shape
        sq = w1.shape[0]
        dev = x.device
        pooled = torch.empty(N, C, dtype=torch.float32, device=dev)
        hpre = torch.empty(N, sq, dtype=torch.float32, device=dev)
        a = torch.empty(N, C, dtype=torch.float32, device=dev)
        y = torch.empty_like(x)
        w1c, w2c = w1.reshape(sq, C).contiguous(), w2.reshape(C, sq).contiguous()
        with timing.region(timing.name("se_fwd", x.shape, "_SqueezeExcite")):
            _lib.call("e2ep_se_fwd", _lib.ptr(x), None, None, _lib.ptr(w1c), _lib.ptr(b1), _lib.ptr(w2c),
                      _lib.ptr(b2), N, C, H * W, sq, _lib.ptr(pooled), _lib.ptr(hpre), _lib.ptr(a),
                      _lib.ptr(y), _lib.stream(), 0)
        ctx.save_for_backward(x, w1c, w2c, pooled, hpre, a)
        ctx.shapes = (w1.shape, w2.shape, b1 is not None, b2 is not None)
        return y

    @staticmethod
    def backward(ctx, dy):
        x, w1c, w2c, pooled, hpre, a = ctx.saved_tensors
        w1s, w2s, hb1, hb2 = ctx.shapes
        N, C, H, W = x.shape
        sq = w1c.shape[0]
        nig = ctx.needs_input_grad
        dev = x.device
        dx = torch.empty_like(x) if nig[0] else None
        dw1 = torch.empty(w1s, dtype=torch.float32, device=dev) if nig[1] else None
        db1 = torch.empty(sq, dtype=torch.float32, device=dev) if (hb1 and nig[2]) else None
        dw2 = torch.empty(w2s, dtype=torch.float32, device=dev) if nig[3] else None
        db2 = torch.empty(C, dtype=torch.float32, device=dev) if (hb2 and nig[4]) else None
        ws = torch.empty(2 * N * C + 17 * N * sq, dtype=torch.float32, device=dev)
        with timing.region(timing.name("se_bwd", x.shape, "_SqueezeExcite")):
            _lib.call("e2ep_se_bwd", _lib.ptr(x), None, None, _lib.ptr(dy.contiguous()),
                      _lib.ptr(w1c), _lib.ptr(w2c), _lib.ptr(pooled), _lib.ptr(hpre), _lib.ptr(a),
                      N, C, H * W, sq, _lib.ptr(dx), None, _lib.ptr(dw1), _lib.ptr(db1), _lib.ptr(dw2), _lib.ptr(db2),
                      _lib.ptr(ws), _lib.stream(), 0)
        return dx, dw1, db1, dw2, db2


# E2EP_BN_SE_SUMS=0: the _bn1 backward takes its own reduction pass (e2ep_bn_bwd) instead of
# the sums from the SE's da pass (A/B)
_SE_BN_SUMS = [os.environ.get("E2EP_BN_SE_SUMS", "1") != "0"]


def set_se_bn_sums(on):
    """Enable / disable the _bn1 backward sums from the SE pass (returns the previous setting)."""
    prev = _SE_BN_SUMS[0]
    _SE_BN_SUMS[0] = bool(on)
    return prev


class _BnSwishSE(torch.autograd.Function):
    """squeeze_excite(batch_norm_act(x, bn, 'swish'), ...) with the BN + swish applied on load
    by the SE kernels (MBConv _bn1 -> swish -> SE, reference model/cam_encoder.py:69-73 via
    efficientnet-pytorch MBConvBlock.forward): the activation tensor is never written, and
    the backward forms its gradient inside the BN backward (gate_logit / gate_dpooled)."""

    @staticmethod
    def forward(ctx, x, gamma, beta, rm, rv, train, momentum, eps, w1, b1, w2, b2, part=None,
                tiles=0, pre=None):
        x = x.contiguous()
        N, C, H, W = x.shape
        sq = w1.shape[0]
        dev = x.device
        f32 = dict(dtype=torch.float32, device=dev)
        stats = pre if pre is not None else torch.empty(4, C, **f32)  # mean, invstd, scale, shift
        s = _lib.stream()
        with timing.region(timing.name("bn_fwd", x.shape, "_BnSwishSE")):
            if pre is not None:  # eval statistics of the forward's EvalBnBatch launch
                pass
            elif part is not None and train:  # partials from the depthwise kernel
                fws = _ws(_lib.load().e2ep_bn_finalize_part_workspace(C, tiles), x.device)
                _lib.call("e2ep_bn_finalize_part", _lib.ptr(part), tiles, _lib.ptr(gamma),
                          _lib.ptr(beta), _lib.ptr(rm), _lib.ptr(rv), N, C, H, W, float(momentum),
                          float(eps), _lib.ptr(stats[0]), _lib.ptr(stats[1]), _lib.ptr(stats[2]),
                          _lib.ptr(stats[3]), _lib.ptr(fws), _lib.nbytes(fws), s)
            else:
                ws = _ws(_lib.load().e2ep_bn_workspace(N, C, H, W), dev)
                _lib.call("e2ep_bn_stats", _lib.ptr(x), _lib.ptr(gamma), _lib.ptr(beta), _lib.ptr(rm),
                          _lib.ptr(rv), N, C, H, W, int(train), float(momentum), float(eps),
                          _lib.ptr(stats[0]), _lib.ptr(stats[1]), _lib.ptr(stats[2]),
                          _lib.ptr(stats[3]), _lib.ptr(ws), _lib.nbytes(ws), s,
                          _IO_X if _is_bf16(x) else 0)
        pooled, hpre, a = torch.empty(N, C, **f32), torch.empty(N, sq, **f32), torch.empty(N, C, **f32)
        # a bf16-stored input (bf16 storage, _store_bf16): at level 2 the output — the project
        # conv's input — is stored bf16 too
        hb = _is_bf16(x)
        yb = hb and _BF16_STORE[0] >= 2  # the output stored bf16 as well (level 2)
        y = torch.empty(x.shape, dtype=torch.bfloat16 if yb else torch.float32, device=dev)
        w1c, w2c = w1.reshape(sq, C).contiguous(), w2.reshape(C, sq).contiguous()
        with timing.region(timing.name("se_fwd", x.shape, "_BnSwishSE")):
            _lib.call("e2ep_se_fwd", _lib.ptr(x), _lib.ptr(stats[2]), _lib.ptr(stats[3]),
                      _lib.ptr(w1c), _lib.ptr(b1), _lib.ptr(w2c), _lib.ptr(b2), N, C, H * W, sq,
                      _lib.ptr(pooled), _lib.ptr(hpre), _lib.ptr(a), _lib.ptr(y), s,
                      (_IO_X | (_IO_DX if yb else 0)) if hb else 0)
        ctx.save_for_backward(x, gamma, beta, stats, w1c, w2c, pooled, hpre, a)
        ctx.shapes = (w1.shape, w2.shape, b1 is not None, b2 is not None)
        ctx.train = train
        return y

    @staticmethod
    def backward(ctx, dy):
        x, gamma, beta, stats, w1c, w2c, pooled, hpre, a = ctx.saved_tensors
        w1s, w2s, hb1, hb2 = ctx.shapes
        N, C, H, W = x.shape
        sq = w1c.shape[0]
        nig = ctx.needs_input_grad
        dev = x.device
        f32 = dict(dtype=torch.float32, device=dev)
        dy = dy.contiguous()
        s = _lib.stream()
        dw1 = torch.empty(w1s, **f32) if nig[8] else None
        db1 = torch.empty(sq, **f32) if (hb1 and nig[9]) else None
        dw2 = torch.empty(w2s, **f32) if nig[10] else None
        db2 = torch.empty(C, **f32) if (hb2 and nig[11]) else None
        dpooled = torch.empty(N, C, **f32)
        ws = torch.empty(2 * N * C + 17 * N * sq, **f32)
        dx = torch.empty_like(x) if nig[0] else None  # bf16 with a bf16-stored x
        dg = torch.empty_like(gamma) if (gamma is not None and nig[1]) else None
        db = torch.empty_like(beta) if (beta is not None and nig[2]) else None
        hb = _is_bf16(x)
        # storage of the incoming gradient (bf16 at a bf16-stored output)
        io_in = (_IO_X | (_IO_DY if _is_bf16(dy) else 0)) if hb else 0
        # training BN on the split path: its channel sums are taken in the SE's da pass
        # (e2ep_se_bwd_bn), so the BN backward is its apply pass alone
        fused = (_SE_BN_SUMS[0] and ctx.train and dx is not None
                 and _lib.load().e2ep_bn_bwd_split(N, C, H, W) == 1)
        if fused:
            planes = torch.empty(N * C * 4, dtype=torch.float64, device=dev)
            with timing.region(timing.name("se_bwd", x.shape, "_BnSwishSE")):
                _lib.call("e2ep_se_bwd_bn", _lib.ptr(x), _lib.ptr(stats[2]), _lib.ptr(stats[3]),
                          _lib.ptr(stats[0]), _lib.ptr(stats[1]), _lib.ptr(gamma), _lib.ptr(beta),
                          _lib.ptr(dy), _lib.ptr(w1c), _lib.ptr(w2c), _lib.ptr(pooled),
                          _lib.ptr(hpre), _lib.ptr(a), N, C, H * W, sq, _lib.ptr(dpooled),
                          _lib.ptr(dw1), _lib.ptr(db1), _lib.ptr(dw2), _lib.ptr(db2),
                          _lib.ptr(planes), _lib.ptr(ws), s, io_in)
            with timing.region(timing.name("bn_bwd", x.shape, "_BnSwishSE")):
                _lib.call("e2ep_bn_bwd_planes", _lib.ptr(x), _lib.ptr(dy), _lib.ptr(stats[0]),
                          _lib.ptr(stats[1]), _lib.ptr(gamma), _lib.ptr(beta), _lib.ptr(a),
                          _lib.ptr(dpooled), _lib.ptr(planes), N, C, H, W, ACT["swish"],
                          _lib.ptr(dx), _lib.ptr(dg), _lib.ptr(db), s, (io_in | _IO_DX) if hb else 0)
            return dx, dg, db, None, None, None, None, None, dw1, db1, dw2, db2, None, None, None
        with timing.region(timing.name("se_bwd", x.shape, "_BnSwishSE")):
            _lib.call("e2ep_se_bwd", _lib.ptr(x), _lib.ptr(stats[2]), _lib.ptr(stats[3]),
                      _lib.ptr(dy), _lib.ptr(w1c), _lib.ptr(w2c), _lib.ptr(pooled),
                      _lib.ptr(hpre), _lib.ptr(a), N, C, H * W, sq, None, _lib.ptr(dpooled),
                      _lib.ptr(dw1), _lib.ptr(db1), _lib.ptr(dw2), _lib.ptr(db2), _lib.ptr(ws), s,
                      io_in)
        if dx is not None or dg is not None or db is not None:
            bws = _ws(_lib.load().e2ep_bn_workspace(N, C, H, W), dev)
            with timing.region(timing.name("bn_bwd", x.shape, "_BnSwishSE")):
                _lib.call("e2ep_bn_bwd", _lib.ptr(x), _lib.ptr(dy), _lib.ptr(stats[0]),
                          _lib.ptr(stats[1]), _lib.ptr(gamma), _lib.ptr(beta), None, None, 1.0,
                          _lib.ptr(a), _lib.ptr(dpooled), N, C, H, W, int(ctx.train), ACT["swish"],
                          _lib.ptr(dx), _lib.ptr(dg), _lib.ptr(db), None, _lib.ptr(bws), _lib.nbytes(bws), s,
                          (io_in | _IO_DX) if hb else 0)
        return dx, dg, db, None, None, None, None, None, dw1, db1, dw2, db2, None, None, None


def bn_swish_squeeze_excite(x, bn, w1, b1, w2, b2):
    """squeeze_excite(batch_norm_act(x, bn, 'swish'), w1, b1, w2, b2) as one fused op."""
    _dev(x)
    train = _bn_train_and_count(bn)
    rm = bn.running_mean if bn.track_running_stats else None
    rv = bn.running_var if bn.track_running_stats else None
    mom = bn.momentum if bn.momentum is not None else 0.1
    pp = conv.bn_partials(x) if train else None
    return _BnSwishSE.apply(x, bn.weight, bn.bias, rm, rv, train, mom, bn.eps, w1, b1, w2, b2,
                            *(pp or (None, 0)), None if train else _eval_bn_stats(bn))


def squeeze_excite(x, w1, b1, w2, b2):
    """x * sigmoid(w2 swish(w1 mean_hw(x) + b1) + b2): efficientnet-pytorch MBConv SE with the
    two 1x1 convs (w1 [sq,C,1,1], w2 [C,sq,1,1]) on the pooled 1x1 map."""
    _dev(x)
    return _SqueezeExcite.apply(x, w1, b1, w2, b2)


# ------------------------------------------------------------------------------------------
# channel concatenation, loss sum, PAD mask (csrc/small.hip)
# ------------------------------------------------------------------------------------------
class _CatChannels(torch.autograd.Function):
    @staticmethod
    def forward(ctx, *xs):
        xs = [x.contiguous() for x in xs]
        N, _, H, W = xs[0].shape
        chans = [x.shape[1] for x in xs]
        y = torch.empty(N, sum(chans), H, W, dtype=torch.float32, device=xs[0].device)
        n = len(xs)
        _lib.call("e2ep_cat_channels", (ctypes.c_void_p * n)(*[x.data_ptr() for x in xs]),
                  (ctypes.c_int * n)(*chans), n, N, H * W, _lib.ptr(y), _lib.stream())
        ctx.chans = chans
        return y

    @staticmethod
    def backward(ctx, g):
        g = g.contiguous()
        N, _, H, W = g.shape
        outs = [torch.empty(N, c, H, W, dtype=torch.float32, device=g.device) for c in ctx.chans]
        n = len(outs)
        _lib.call("e2ep_split_channels", _lib.ptr(g), (ctypes.c_int * n)(*ctx.chans), n, N, H * W,
                  (ctypes.c_void_p * n)(*[o.data_ptr() for o in outs]), _lib.stream())
        return tuple(outs)


def cat_channels(xs):
    """torch.cat(xs, 1) of NCHW fp32 device tensors as one e2ep launch, and its backward as
    one launch writing every piece's gradient contiguous (no slice copies downstream).  Falls
    back to torch.cat outside the kernel's range (more than 8 pieces, H*W % 4 != 0)."""
    _dev(*xs)
    if (len(xs) > 8 or any(x.dim() != 4 or x.dtype != torch.float32 for x in xs)
            or (xs[0].shape[2] * xs[0].shape[3]) % 4):
        return torch.cat(xs, 1)
    return _CatChannels.apply(*xs)


class _Transpose12(torch.autograd.Function):
    """(B, R, C) -> (B, C, R) contiguous with e2ep_transpose each way."""

    @staticmethod
    def forward(ctx, x):
        x = x.contiguous()
        B, R, C = x.shape
        out = torch.empty(B, C, R, dtype=torch.float32, device=x.device)
        _lib.call("e2ep_transpose", _lib.ptr(x), R * C, B, R, C, _lib.ptr(out), _lib.stream())
        return out

    @staticmethod
    def backward(ctx, g):
        g = g.contiguous()
        B, C, R = g.shape
        dx = torch.empty(B, R, C, dtype=torch.float32, device=g.device)
        _lib.call("e2ep_transpose", _lib.ptr(g), R * C, B, C, R, _lib.ptr(dx), _lib.stream())
        return dx


def transpose12(x):
    """x.transpose(1, 2).contiguous() of a (B, R, C) fp32 device tensor, one e2ep launch each
    way (the fusion tokens -> BEV map hand-off to the segmentation head)."""
    _dev(x)
    return _Transpose12.apply(x)


class _Fork2(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x):
        return x.view_as(x), x.view_as(x)

    @staticmethod
    def backward(ctx, g1, g2):
        if g1 is None or g2 is None:
            return g2 if g1 is None else g1
        g1, g2 = g1.contiguous(), g2.contiguous()
        out = torch.empty_like(g1)
        _lib.call("e2ep_add_f32", _lib.ptr(g1), _lib.ptr(g2), g1.numel(), _lib.ptr(out),
                  _lib.stream())
        return out


def fork2(x):
    """Two handles of x for two consumers; their gradients are summed by one e2ep launch
    (autograd would sum them with a PyTorch add kernel)."""
    _dev(x)
    return _Fork2.apply(x)


class _Sum3(torch.autograd.Function):
    @staticmethod
    def forward(ctx, a, b, c):
        out = torch.empty((), dtype=torch.float32, device=a.device)
        _lib.call("e2ep_sum3", _lib.ptr(a), _lib.ptr(b), _lib.ptr(c), _lib.ptr(out), _lib.stream())
        return out

    @staticmethod
    def backward(ctx, g):
        return g, g, g


def sum3(a, b, c):
    """(a + b) + c of three fp32 device scalars in one launch (the step's total loss)."""
    _dev(a, b, c)
    return _Sum3.apply(a, b, c)


def eq_mask(tok, value):
    """tok == value for a (B, T) int64 device tensor with unit column stride, as a bool mask
    (one launch)."""
    if tok.dtype != torch.int64 or tok.dim() != 2 or tok.stride(1) != 1 or not tok.is_cuda:
        raise _lib.E2EPError("eq_mask: (B, T) int64 device tensor with unit column stride")
    B, T = tok.shape
    m = torch.empty(B, T, dtype=torch.bool, device=tok.device)
    _lib.call("e2ep_eq_mask_i64", _lib.ptr(tok), tok.stride(0), B, T, int(value), _lib.ptr(m),
              _lib.stream())
    return m


# ------------------------------------------------------------------------------------------
# residual add + dropout + LayerNorm (post-norm transformer layers)
# ------------------------------------------------------------------------------------------
class _AddDropLN(torch.autograd.Function):
    @staticmethod
    def forward(ctx, a, b, gamma, beta, u, seed, p, eps):
        a = a.contiguous()
        b = b.contiguous()
        E = a.shape[-1]
        rows = a.numel() // E
        x = torch.empty_like(a)
        y = torch.empty_like(a)
        mean = torch.empty(rows, dtype=torch.float32, device=a.device)
        rstd = torch.empty_like(mean)
        # mask from `u` (explicit uniforms) or, without u, from the counter hash keyed by seed
        fn, mask = ("e2ep_add_drop_ln_fwd", u) if seed is None else ("e2ep_add_drop_ln_fwd_seeded", seed)
        with timing.region(timing.name("ln_fwd", a.shape, "_AddDropLN")):
            _lib.call(fn, _lib.ptr(a), _lib.ptr(b), _lib.ptr(mask), float(p),
                      _lib.ptr(gamma), _lib.ptr(beta), rows, E, float(eps), _lib.ptr(x), _lib.ptr(y),
                      _lib.ptr(mean), _lib.ptr(rstd), _lib.stream())
        ctx.save_for_backward(x, mean, rstd, gamma, mask)
        ctx.p, ctx.rows, ctx.E, ctx.seeded = float(p), rows, E, seed is not None
        return y

    @staticmethod
    def backward(ctx, dy):
        x, mean, rstd, gamma, mask = ctx.saved_tensors
        nig = ctx.needs_input_grad
        da = torch.empty_like(x) if nig[0] else None
        db = torch.empty_like(x) if nig[1] else None
        dg = torch.empty_like(gamma) if (gamma is not None and nig[2]) else None
        dbeta = torch.empty_like(gamma) if (gamma is not None and nig[3]) else None
        ws = _ws(_lib.load().e2ep_add_drop_ln_bwd_workspace(ctx.rows, ctx.E), x.device)
        with timing.region(timing.name("ln_bwd", x.shape, "_AddDropLN")):
            _lib.call("e2ep_add_drop_ln_bwd_seeded" if ctx.seeded else "e2ep_add_drop_ln_bwd",
                      _lib.ptr(dy.contiguous()), _lib.ptr(x), _lib.ptr(mean),
                      _lib.ptr(rstd), _lib.ptr(gamma), _lib.ptr(mask), ctx.p, ctx.rows, ctx.E,
                      _lib.ptr(da), _lib.ptr(db), _lib.ptr(dg), _lib.ptr(dbeta), _lib.ptr(ws),
                      _lib.stream())
        return da, db, dg, dbeta, None, None, None, None


def add_drop_layer_norm(a, b, norm, p=0.0, u=None, seed=None):
    """norm(a + dropout_p(b)) for an nn.LayerNorm `norm` over the last dim, one fused op.
    The dropout mask is [u >= p] when uniforms `u` are given, else the counter hash keyed by a
    device seed (e2ep_amd.rng: this step's pool; graph-capturable, nothing drawn per element)."""
    _dev(a, b)
    if p > 0.0 and u is None and seed is None:
        seed = rng.seed(a.device)
    if p == 0.0:
        u = seed = None
    return _AddDropLN.apply(a, b, norm.weight, norm.bias, u, seed, p, norm.eps)


# ------------------------------------------------------------------------------------------
# nn.Linear on e2ep_gemm (forward, input gradient, weight gradient) + e2ep_col_sum (bias grad)
# ------------------------------------------------------------------------------------------
def gemm(A, a_kcontig, B, b_kcontig, M, N, K, bias=None, cadd=None, out=None, relu=False,
         tag="gemm", ws=None):
    """C (M x N, row-major) = A(m,k) B(k,n) (+ bias[n]) (+ cadd) (ReLU) on e2ep_gemm.
    A is (M x K) when a_kcontig else (K x M), B is (N x K) when b_kcontig else (K x N); both
    row-major with unit inner stride."""
    for t, n in ((A, "A"), (B, "B")):
        if t.dim() != 2 or t.stride(1) != 1 or t.dtype != torch.float32:
            raise _lib.E2EPError(f"gemm: {n} must be a 2-D fp32 matrix with unit inner stride")
    want_a = (M, K) if a_kcontig else (K, M)
    want_b = (N, K) if b_kcontig else (K, N)
    if tuple(A.shape) != want_a or tuple(B.shape) != want_b:
        raise _lib.E2EPError(f"gemm: A {tuple(A.shape)} / B {tuple(B.shape)} vs M={M} N={N} K={K}")
    if out is None:
        out = torch.empty(M, N, dtype=torch.float32, device=A.device)
    if cadd is not None and (cadd.shape != (M, N) or cadd.stride(1) != 1):
        raise _lib.E2EPError("gemm: cadd must be (M, N) with unit inner stride")
    if ws is None:
        ws = _ws(_lib.load().e2ep_gemm_workspace(M, N, K), A.device)
    with timing.region(timing.name("gemm", (M, N, K), tag), 2.0 * M * N * K):
        _lib.call("e2ep_gemm", _lib.ptr(A), A.stride(0), int(a_kcontig), _lib.ptr(B), B.stride(0),
                  int(b_kcontig), _lib.ptr(bias), _lib.ptr(cadd),
                  cadd.stride(0) if cadd is not None else 0, _lib.ptr(out), out.stride(0), M, N, K,
                  int(relu), _lib.ptr(ws), _lib.nbytes(ws), _lib.stream())
    return out


class _Linear(torch.autograd.Function):
    """y = x W^T + b (+ ReLU).  All three GEMMs are e2ep_gemm: forward (bias and ReLU in the
    epilogue), dX = dY W (the residual's gradient added in the epilogue when skip is used),
    dW = dY^T X with the bias gradient as the same launch's row sum (e2ep_gemm_rowsum); without
    a weight gradient the bias gradient is e2ep_col_sum."""

    @staticmethod
    def forward(ctx, x, weight, bias, skip=False, relu=False):
        K = x.shape[-1]
        x2 = x.reshape(-1, K)
        if x2.stride(1) != 1 or x2.stride(0) != K:
            x2 = x2.contiguous()
        N = weight.shape[0]
        y = gemm(x2, True, weight, True, x2.shape[0], N, K, bias=bias, relu=relu, tag="linear_fwd")
        ctx.save_for_backward(x2, weight, y if relu else None)
        ctx.has_bias, ctx.relu, ctx.xshape = bias is not None, relu, x.shape
        y = y.view(*x.shape[:-1], N)
        # skip: also hand x back for the layer's residual connection; that gradient is then
        # accumulated by the input-gradient GEMM's epilogue, not by an autograd add
        return (y, x) if skip else y

    @staticmethod
    def backward(ctx, gy, gskip=None):
        x2, weight, y = ctx.saved_tensors
        nig = ctx.needs_input_grad
        M, K = x2.shape
        N = weight.shape[0]
        g2 = gy.reshape(M, N)
        if g2.stride(1) != 1 or g2.stride(0) != N:
            g2 = g2.contiguous()
        if ctx.relu:  # dY * [y > 0] (relu derivative on the output), one e2ep launch
            gr = torch.empty_like(g2)
            _lib.call("e2ep_act_bwd", _lib.ptr(y), _lib.ptr(g2), g2.numel(), 1, _lib.ptr(gr),
                      _lib.stream())
            g2 = gr
        dx, dw, db = _linear_bwd(g2, x2, weight, nig[0], nig[1], ctx.has_bias and nig[2], gskip)
        return (dx.view(ctx.xshape) if dx is not None else None), dw, db, None, None


# E2EP_LINEAR_PAIR=0: a linear backward as two launches on forked streams (A/B timing)
_PAIR = [os.environ.get("E2EP_LINEAR_PAIR", "1") != "0"]


def _linear_bwd(g2, x2, weight, want_x, want_w, want_b, gskip=None, dw=None, db=None):
    """Gradients of y2 = x2 W^T + b from g2 = dY2 (M x N): dX2 = g2 W (+ gskip in the
    epilogue), dW = g2^T x2 with db = row sums of g2^T in the same launch (e2ep_gemm_rowsum),
    db alone by e2ep_col_sum.  dw / db may be given (row slices of a larger gradient)."""
    M, K = x2.shape
    N = weight.shape[0]
    dx = None
    if want_x and want_w and want_b and _PAIR[0]:
        # all three in one launch (e2ep_linear_bwd: k_gemm_pair), no side-stream fork / join
        if dw is None:
            dw = torch.empty(N, K, dtype=torch.float32, device=g2.device)
        if db is None:
            db = torch.empty(N, dtype=torch.float32, device=g2.device)
        cadd = gskip.reshape(M, K) if gskip is not None else None
        if cadd is not None and cadd.stride(1) != 1:
            cadd = cadd.contiguous()
        dx = torch.empty(M, K, dtype=torch.float32, device=g2.device)
        lib = _lib.load()
        wsx = _ws(lib.e2ep_gemm_workspace(M, K, N), g2.device)
        wsw = _ws(lib.e2ep_gemm_rowsum_workspace(N, K, M), g2.device)
        w2 = weight if weight.stride(1) == 1 else weight.contiguous()
        with timing.region(timing.name("gemm", (M, N, K), "linear_bwd_pair"), 4.0 * M * N * K):
            _lib.call("e2ep_linear_bwd", _lib.ptr(g2), g2.stride(0), _lib.ptr(x2), x2.stride(0),
                      _lib.ptr(w2), w2.stride(0), _lib.ptr(cadd),
                      cadd.stride(0) if cadd is not None else 0, _lib.ptr(dx), dx.stride(0),
                      _lib.ptr(dw), dw.stride(0), _lib.ptr(db), M, N, K, _lib.ptr(wsx),
                      _lib.nbytes(wsx), _lib.ptr(wsw), _lib.nbytes(wsw), _lib.stream())
        return dx, dw, db
    # weight / bias gradients on the side stream, concurrent with the input gradient
    # (conv._Fork: every buffer allocated here, on the current stream, before the fork)
    fork = None
    if want_w or want_b:
        if want_w:
            if dw is None:
                dw = torch.empty(N, K, dtype=torch.float32, device=g2.device)
            wsw = _ws(_lib.load().e2ep_gemm_rowsum_workspace(N, K, M) if want_b
                      else _lib.load().e2ep_gemm_workspace(N, K, M), g2.device)
        if want_b:
            if db is None:
                db = torch.empty(N, dtype=torch.float32, device=g2.device)
            wsb = None if want_w else _ws(_lib.load().e2ep_col_sum_workspace(M, N), g2.device)
        fork = conv._Fork(g2.device, on=want_x, work_us=conv.est_us(2.0 * N * K * M))
        with fork:
            if want_w and want_b:  # dW and db in one launch
                with timing.region(timing.name("gemm", (N, K, M), "linear_wgrad"), 2.0 * N * K * M):
                    _lib.call("e2ep_gemm_rowsum", _lib.ptr(g2), g2.stride(0), _lib.ptr(x2),
                              x2.stride(0), _lib.ptr(dw), dw.stride(0), _lib.ptr(db), N, K, M,
                              _lib.ptr(wsw), _lib.nbytes(wsw), _lib.stream())
            elif want_w:
                gemm(g2, False, x2, False, N, K, M, out=dw, ws=wsw, tag="linear_wgrad")
            else:
                _lib.call("e2ep_col_sum", _lib.ptr(g2), M, N, _lib.ptr(db), _lib.ptr(wsb),
                          _lib.stream())
    if want_x:
        cadd = gskip.reshape(M, K) if gskip is not None else None
        if cadd is not None and cadd.stride(1) != 1:
            cadd = cadd.contiguous()
        dx = gemm(g2, True, weight, False, M, K, N, cadd=cadd, tag="linear_dgrad")
    if fork is not None:
        fork.join()
    return dx, (dw if want_w else None), (db if want_b else None)


def _rows2(x):
    K = x.shape[-1]
    x2 = x.reshape(-1, K)
    return x2 if (x2.stride(1) == 1 and x2.stride(0) == K) else x2.contiguous()


class _InProjQKV(torch.autograd.Function):
    """Cross-attention in-projection with one weight [3E, E] (nn.MultiheadAttention's
    in_proj_weight / in_proj_bias): q = xq Wq^T + bq, kv = xkv Wkv^T + bkv with Wq = W[:E],
    Wkv = W[E:], and xq handed back for the layer's residual (its gradient joins dxq in the
    GEMM epilogue).  The backward writes dW / db row blocks straight into one [3E, E] / [3E]
    gradient, so no split-backward concatenation runs."""

    @staticmethod
    def forward(ctx, xq, xkv, weight, bias, E):
        xq2, xkv2 = _rows2(xq), _rows2(xkv)
        K = xq2.shape[1]
        Wq, Wkv = weight[:E], weight[E:]
        bq, bkv = (None, None) if bias is None else (bias[:E], bias[E:])
        q = gemm(xq2, True, Wq, True, xq2.shape[0], E, K, bias=bq, tag="linear_fwd")
        kv = gemm(xkv2, True, Wkv, True, xkv2.shape[0], 2 * E, K, bias=bkv, tag="linear_fwd")
        ctx.save_for_backward(xq2, xkv2, weight)
        ctx.E, ctx.has_bias, ctx.shapes = E, bias is not None, (xq.shape, xkv.shape)
        ctx.set_materialize_grads(False)  # unused aliases (the last layer's memory) stay None
        return q.view(*xq.shape[:-1], E), kv.view(*xkv.shape[:-1], 2 * E), xq, xkv

    @staticmethod
    def backward(ctx, gq, gkv, gskip, gskip_kv):
        xq2, xkv2, weight = ctx.saved_tensors
        nig = ctx.needs_input_grad
        E = ctx.E
        want_b = ctx.has_bias and nig[3]
        dw = torch.empty_like(weight) if nig[2] else None
        db = torch.empty(3 * E, dtype=torch.float32, device=weight.device) if want_b else None
        dxq, _, _ = _linear_bwd(_rows2(gq), xq2, weight[:E], nig[0], nig[2], want_b, gskip,
                                dw[:E] if dw is not None else None,
                                db[:E] if db is not None else None)
        dxkv, _, _ = _linear_bwd(_rows2(gkv), xkv2, weight[E:], nig[1], nig[2], want_b, gskip_kv,
                                 dw[E:] if dw is not None else None,
                                 db[E:] if db is not None else None)
        sq, skv = ctx.shapes
        return (dxq.view(sq) if dxq is not None else None,
                dxkv.view(skv) if dxkv is not None else None, dw, db, None)


def in_proj_qkv(xq, xkv, weight, bias, E):
    """(q, kv, xq_skip, xkv_skip) of a cross-attention in-projection (see _InProjQKV):
    xkv_skip carries the key/value input on to another consumer (the next decoder layer's
    memory), its gradient joining dxkv in the GEMM epilogue."""
    _dev(xq, xkv, weight, bias)
    return _InProjQKV.apply(xq, xkv, weight, bias, int(E))


def linear(x, weight, bias=None, skip=False, relu=False):
    """F.linear(x, weight, bias) (then ReLU when relu) on e2ep_gemm, fp32 HIP tensors.
    skip=True returns (y, x_skip): use x_skip for the residual connection around this layer
    and its gradient joins dx inside the GEMM epilogue."""
    _dev(x, weight, bias)
    if x.dtype != torch.float32 or weight.dtype != torch.float32 or weight.stride(-1) != 1:
        raise _lib.E2EPError("linear: fp32 input and a weight with unit inner stride required")
    return _Linear.apply(x, weight, bias, bool(skip), bool(relu))


# ------------------------------------------------------------------------------------------
# transformer feed-forward activation: dropout_p(relu(x))
# ------------------------------------------------------------------------------------------
class _ReluDropout(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, p, seed):
        y = torch.empty_like(x)
        _lib.call("e2ep_relu_dropout_fwd", _lib.ptr(x), x.numel(), float(p), _lib.ptr(seed),
                  _lib.ptr(y), _lib.stream())
        ctx.save_for_backward(x, seed)
        ctx.p = float(p)
        return y

    @staticmethod
    def backward(ctx, dy):
        x, seed = ctx.saved_tensors
        dy = dy.contiguous()
        dx = torch.empty_like(x)
        _lib.call("e2ep_relu_dropout_bwd", _lib.ptr(x), _lib.ptr(dy), x.numel(), ctx.p,
                  _lib.ptr(seed), _lib.ptr(dx), _lib.stream())
        return dx, None, None


def relu_dropout(x, p=0.0, seed=None):
    """dropout_p(relu(x)) as one e2ep launch each way (fp32 HIP tensor, numel % 4 == 0).
    The mask is a hash of a per-call device seed (drawn here when p > 0 and none is given:
    graph-capturable) and the element index."""
    _dev(x)
    x = x.contiguous()
    if p > 0.0 and seed is None:
        seed = rng.seed(x.device)
    return _ReluDropout.apply(x, float(p), seed)


# ------------------------------------------------------------------------------------------
# transformer token assembly + positional embedding + pos_drop (csrc/tokens.hip)
# ------------------------------------------------------------------------------------------
class _FusionTokens(torch.autograd.Function):
    @staticmethod
    def forward(ctx, bev, motion, pos, p, seed):
        B, C, S = bev.shape
        E = pos.shape[-1]
        out = torch.empty((B, S, E), dtype=torch.float32, device=bev.device)
        _lib.call("e2ep_fusion_tokens_fwd", _lib.ptr(bev), _lib.ptr(motion), _lib.ptr(pos), B, C, S,
                  E, float(p), _lib.ptr(seed), _lib.ptr(out), _lib.stream())
        ctx.save_for_backward(seed)
        ctx.meta = (B, C, S, E, float(p), tuple(motion.shape))
        return out

    @staticmethod
    def backward(ctx, g):
        (seed,) = ctx.saved_tensors
        B, C, S, E, p, mshape = ctx.meta
        g = g.contiguous()
        dbev = torch.empty((B, C, S), dtype=torch.float32, device=g.device)
        dmotion = torch.empty(mshape, dtype=torch.float32, device=g.device)
        dpos = torch.empty((1, S, E), dtype=torch.float32, device=g.device)
        _lib.call("e2ep_fusion_tokens_bwd", _lib.ptr(g), B, C, S, E, p, _lib.ptr(seed),
                  _lib.ptr(dbev), _lib.ptr(dmotion), _lib.ptr(dpos), _lib.stream())
        return dbev, dmotion, dpos, None, None


def fusion_tokens(bev, motion, pos, p=0.0, seed=None):
    """drop(cat([bev.transpose(1, 2), motion.transpose(1, 2).expand(-1, -1, E - C)], 2) + pos)
    in one launch each way (reference model/feature_fusion.py:41-46): bev (B, C, S), motion
    (B, 1, S), pos (1, S, E) fp32 HIP tensors."""
    _dev(bev, motion, pos)
    bev, motion, pos = bev.contiguous(), motion.contiguous(), pos.contiguous()
    if p > 0.0 and seed is None:
        seed = rng.seed(bev.device)
    return _FusionTokens.apply(bev, motion, pos, float(p), seed)


class _EmbedTokens(torch.autograd.Function):
    @staticmethod
    def forward(ctx, tok, table, pos, p, seed):
        B, T = tok.shape
        V, E = table.shape
        out = torch.empty((B, T, E), dtype=torch.float32, device=table.device)
        _lib.call("e2ep_embed_tokens_fwd", _lib.ptr(tok), tok.stride(0), _lib.ptr(table), V,
                  _lib.ptr(pos), B, T, E, float(p), _lib.ptr(seed), _lib.ptr(out), _lib.stream())
        ctx.save_for_backward(tok, seed)
        ctx.meta = (B, T, V, E, float(p))
        return out

    @staticmethod
    def backward(ctx, g):
        tok, seed = ctx.saved_tensors
        B, T, V, E, p = ctx.meta
        g = g.contiguous()
        dtable = torch.empty((V, E), dtype=torch.float32, device=g.device)
        dpos = torch.empty((1, T, E), dtype=torch.float32, device=g.device)
        _lib.call("e2ep_embed_tokens_bwd", _lib.ptr(g), _lib.ptr(tok), tok.stride(0), V, B, T, E, p,
                  _lib.ptr(seed), _lib.ptr(dtable), _lib.ptr(dpos), _lib.stream())
        return None, dtable, dpos, None, None


def embed_tokens(tok, table, pos, p=0.0, seed=None):
    """drop(embedding(tok) + pos) in one launch each way (reference model/control_predict.py:
    53-54): tok (B, T) int64 (row stride free, unit column stride), table (V, E), pos (1, T, E)."""
    _dev(table, pos)
    if tok.dtype != torch.int64 or tok.dim() != 2 or tok.stride(1) != 1 or tok.device != table.device:
        raise _lib.E2EPError("embed_tokens: tok must be a (B, T) int64 device tensor with unit column stride")
    pos = pos.contiguous()
    if tok.numel() and not torch.cuda.is_current_stream_capturing():
        # nn.Embedding raises on an id outside [0, V) (a wrong token_nums or PAD arithmetic);
        # the kernels clamp only for memory safety, so check here, outside captures (a
        # captured step checks its tokens in the eager warm-up steps)
        lo, hi = (int(v) for v in torch.aminmax(tok))
        if lo < 0 or hi >= table.shape[0]:
            raise IndexError(f"embed_tokens: token id out of range [0, {table.shape[0]}): "
                             f"min {lo}, max {hi}")
    if p > 0.0 and seed is None:
        seed = rng.seed(table.device)
    return _EmbedTokens.apply(tok, table, pos, float(p), seed)


# ------------------------------------------------------------------------------------------
# softmax over channels (depth distribution)
# ------------------------------------------------------------------------------------------
class _SoftmaxC(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x):
        x = x.contiguous()
        N, C = x.shape[:2]
        HW = x.numel() // (N * C)
        y = torch.empty_like(x)
        _lib.call("e2ep_softmax_c_fwd", _lib.ptr(x), N, C, HW, _lib.ptr(y), _lib.stream())
        ctx.save_for_backward(y)
        return y

    @staticmethod
    def backward(ctx, dy):
        (y,) = ctx.saved_tensors
        N, C = y.shape[:2]
        HW = y.numel() // (N * C)
        dx = torch.empty_like(y)
        _lib.call("e2ep_softmax_c_bwd", _lib.ptr(y), _lib.ptr(dy.contiguous()), N, C, HW,
                  _lib.ptr(dx), _lib.stream())
        return dx


def softmax_channels(x):
    """x.softmax(dim=1) for an fp32 NC... HIP tensor, one e2ep launch each way."""
    _dev(x)
    return _SoftmaxC.apply(x)
