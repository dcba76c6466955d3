"""Convolution autograd op over the e2ep implicit-GEMM kernels (csrc/conv.hip).

conv2d(x, w, b, stride, padding(l,r,t,b), dilation, act, grad_channels) -> y, backward via
e2ep_conv_dgrad (stride-phase split) / e2ep_conv_wgrad (split pixel reduction) /
e2ep_bias_grad.  1x1 convs on 1x1 maps run on e2ep_skinny_gemm.  groups must be 1
(depthwise convs use e2ep_amd.nn_ops).  `grad_channels` limits the input gradient to the
first channels (the BEV encoder's target-point channel is a constant: no gradient)."""
import os

import torch

from . import _lib, streams, timing


def _ws(nbytes, device):
    return torch.empty(nbytes // 4, dtype=torch.float32, device=device) if nbytes else None


def _rname(kind, dims, extra=""):
    """Timing-region name: per shape when E2EP_TIMING_DETAIL=1 (scripts/conv_breakdown.py)."""
    return f"{kind}{tuple(dims)}{extra}" if timing.detail() else kind


def conv_flops(dims, in_channels=None):
    """Algorithmic FLOPs of one conv launch (fwd, or dgrad / wgrad over in_channels):
    2 * N * Cout * P * Q * Cin * R * S."""
    N, Cin, H, W, Cout, R, S, P, Q = dims[:9]
    return 2.0 * N * Cout * P * Q * (in_channels or Cin) * R * S


class TapMajorBatch:
    """Every spatial conv weight's tap-major copy in one launch per forward.

    The first forward inside the scope transposes per weight (one launch each) and records
    the weights in call order; later forwards transpose all recorded weights with a single
    e2ep_transpose_multi launch at scope entry into persistent buffers (stable addresses, so
    a HIP-graph capture of the step replays it) and tap_major() hands out views.  A weight
    that was not recorded, or whose storage moved (re-flattened parameters), falls back to
    its own launch; a moved weight re-records on the next forward."""

    def __init__(self):
        self.recorded = None   # weights in call order
        self._log = None
        self._views = {}       # id(weight) -> tap-major view, valid while active
        self._key = None
        self._table = None
        self._buf = None
        self._tiles = 0
        self.active = False

    def _build(self, ws):
        dev = ws[0].device
        sizes = [w.numel() for w in ws]
        self._buf = torch.empty(sum(sizes), dtype=torch.float32, device=dev)
        rows, off, tile0 = [], 0, 0
        views = []
        for w, n in zip(ws, sizes):
            Cout, Cin, R, S = w.shape
            v = self._buf[off:off + n].view(R * S, Cout, Cin)
            r, c = Cout * Cin, R * S
            ct = (c + 63) // 64
            rows.append([w.data_ptr(), v.data_ptr(), r, c, tile0, ct])
            tile0 += ((r + 63) // 64) * ct
            off += n
            views.append(v)
        self._table = torch.tensor(rows, dtype=torch.int64).to(dev)
        self._tiles = tile0
        self._key = [(w.data_ptr(), tuple(w.shape)) for w in ws]
        self._vlist = views

    def __enter__(self):
        ws = self.recorded
        if ws is None:
            self._log = []
        elif [(w.data_ptr(), tuple(w.shape)) for w in ws] != self._key:
            self.recorded, self._log = None, []  # storage moved: record again
        else:
            _lib.call("e2ep_transpose_multi", _lib.ptr(self._table), len(ws), self._tiles,
                      _lib.stream())
            self._views = {id(w): v for w, v in zip(ws, self._vlist)}
        self.active = True
        _TAP_BATCH.append(self)
        return self

    def __exit__(self, *exc):
        _TAP_BATCH.pop()
        self.active = False
        self._views = {}
        # the table is built outside any graph capture (a host->device copy): a capture-only
        # process records again on its first eager forward
        if (self.recorded is None and self._log is not None and not exc[0]
                and not torch.cuda.is_current_stream_capturing()):
            log = [w for w in self._log if w.dtype == torch.float32 and w.is_contiguous()]
            if 0 < len(log) <= 256:
                self.recorded = log
                self._build(log)
        self._log = None
        return False

    def lookup(self, w):
        v = self._views.get(id(w))
        if v is None and self._log is not None and all(w is not o for o in self._log):
            self._log.append(w)
        return v


_TAP_BATCH = []  # active TapMajorBatch scopes (innermost last)


def tap_major(w):
    """[Cout,Cin,R,S] -> [R*S,Cout,Cin] (the kernels' w_layout 1); 1x1 filters unchanged."""
    Cout, Cin, R, S = w.shape
    if R * S == 1:
        return w.contiguous()
    if _TAP_BATCH:
        v = _TAP_BATCH[-1].lookup(w)
        if v is not None:
            return v
    out = torch.empty(R * S, Cout, Cin, dtype=torch.float32, device=w.device)
    _lib.call("e2ep_transpose", _lib.ptr(w.contiguous()), Cout * Cin * R * S, 1, Cout * Cin, R * S,
              _lib.ptr(out), _lib.stream())
    return out


# bf16 activation storage (e2ep.h E2EP_IO_*; nn_ops._store_bf16): a bf16 input of a conv (the
# MBConv project conv reading the bf16-stored squeeze-excitation output, C3) is read as bf16 by
# the bf16-operand kernels, and its data gradient is written bf16
_IO_X, _IO_DX = 1, 4


def _io_x(x):
    return _IO_X if x.dtype == torch.bfloat16 else 0


def conv_fwd(x, w, b, dims, act, y, w_layout=0, stats=None):
    """Launch the forward conv into y (handles the split-K workspace).  stats: an fp64 buffer
    for the BatchNorm partial sums of y (e2ep_conv_fwd_stats; see conv2d(bn_stats=True))."""
    d = _lib.dims(dims)
    ws = _ws(_lib.load().e2ep_conv_fwd_workspace(d), x.device)
    with timing.region(_rname("conv_fwd", dims), conv_flops(dims)):
        if stats is None:
            _lib.call("e2ep_conv_fwd", _lib.ptr(x), _lib.ptr(w), _lib.ptr(b), d, act, w_layout,
                      _lib.ptr(y), _lib.ptr(ws), _lib.nbytes(ws), _lib.stream(), _io_x(x))
        else:
            _lib.call("e2ep_conv_fwd_stats", _lib.ptr(x), _lib.ptr(w), _lib.ptr(b), d, act, w_layout,
                      _lib.ptr(y), _lib.ptr(ws), _lib.nbytes(ws), _lib.ptr(stats),
                      _lib.nbytes(stats), _lib.stream(), _io_x(x))
    return y


# E2EP_NO_BN_STATS=1: BN layers compute their own statistics (A/B timing of the epilogue
# statistics; conv2d / depthwise_conv2d then ignore bn_stats=True)
_BN_STATS = [os.environ.get("E2EP_NO_BN_STATS", "0") in ("", "0")]


def bn_partials(y):
    """(partials, tiles) of y's BatchNorm statistics when the conv that produced y wrote them
    (conv2d(bn_stats=True)), else None."""
    return getattr(y, "_e2ep_bn_part", None)


def conv_dgrad(gy, w, dims, m_channels, dx, w_layout=0, res=None):
    """dx = data gradient (+ res, a residual gradient in dx's layout, added in the epilogue);
    a bf16 dx is written bf16."""
    d = _lib.dims(dims)
    ws = _ws(_lib.load().e2ep_conv_dgrad_workspace(d, m_channels), gy.device)
    with timing.region(_rname("conv_dgrad", dims, f"gc{m_channels}"), conv_flops(dims, m_channels)):
        _lib.call("e2ep_conv_dgrad_acc", _lib.ptr(gy), _lib.ptr(w), d, m_channels, w_layout,
                  _lib.ptr(res), _lib.ptr(dx), _lib.ptr(ws), _lib.nbytes(ws), _lib.stream(),
                  _IO_DX if dx.dtype == torch.bfloat16 else 0)
    return dx


def conv_wgrad(gy, x, dims, dw, ws=None):
    d = _lib.dims(dims)
    splits = _lib.load().e2ep_conv_wgrad_splits(d)
    if ws is None:
        ws = torch.empty(splits * dw.numel(), dtype=torch.float32, device=gy.device)
    with timing.region(_rname("conv_wgrad", dims), conv_flops(dims)):
        _lib.call("e2ep_conv_wgrad", _lib.ptr(gy), _lib.ptr(x), d, splits, _lib.ptr(ws), _lib.nbytes(ws),
                  _lib.ptr(dw), 0, _lib.stream(), _io_x(x))
    return dw


# Weight gradients on a side stream.  A conv's weight gradient (and bias gradient) does not
# feed the rest of the backward, so it is launched on a second stream forked from the current
# one and runs concurrently with the data gradient; the current stream joins the side stream
# before the backward returns.  Every tensor the side stream touches is allocated on the
# current stream and still referenced at the join, so the caching allocator cannot hand its
# memory out while the side stream uses it.  Under HIP-graph capture the fork / join become
# parallel graph branches.  Small convs (16x16 / 32x32 maps) fill a fraction of the chip, so
# their two GEMMs overlap instead of running back to back.
#
# A fork is not free in a replayed HIP graph: the side branch starts ~5 us after its fork
# point and the node after the join waits ~9-10 us for the other queue's completion signal
# (scripts/step_sequence.py over the C2 step: 205 idle gaps of 4-10 us, 2.0 ms per step, one
# per fork / join of the transformer's and the 16x16 stages' small layers).  A backward forks
# only when its side work is estimated at >= E2EP_FORK_MIN_US microseconds; shorter pairs run
# back to back on the current stream.  est_us() gives the estimate from the work the caller
# passes (FLOPs at a nominal 40 TF/s, or bytes at 3 TB/s).  Measured (profiles/r04/
# fork_min_us_ab.txt): C2 23.49 / 23.42 / 23.53 / 23.79 / 24.17 / 23.50 ms at 0 / 10 / 20 / 40 /
# 80 us / never — the gaps and the overlap cancel — and C3 20.32 / 20.46 / 20.76 ms at 0 / 20 /
# never, so the default stays 0 (every fork).
_SIDE = {}
_OVERLAP = [os.environ.get("E2EP_WGRAD_OVERLAP", "1") != "0"]
_FORK_MIN_US = [float(os.environ.get("E2EP_FORK_MIN_US", "0"))]


def est_us(flops=0.0, nbytes=0.0):
    """Nominal duration (us) of side-stream work: FLOPs at 40 TF/s plus bytes at 3 TB/s."""
    return flops / 4e7 + nbytes / 3e6


def set_fork_min_us(us):
    """Minimum estimated side work (us) for a fork (returns the previous value)."""
    prev = _FORK_MIN_US[0]
    _FORK_MIN_US[0] = float(us)
    return prev


def set_wgrad_overlap(on):
    """Enable / disable the side-stream weight gradients (returns the previous setting)."""
    prev = _OVERLAP[0]
    _OVERLAP[0] = bool(on)
    return prev


def wgrad_overlap():
    return _OVERLAP[0]


# E2EP_WGRAD_STREAM=cam | heads: the weight-gradient forks of the main stream run on that model
# branch's stream (streams.py) instead of a stream of their own, so a captured train step uses
# three streams instead of four.  With four, the replayed graph idled 0.2 - 0.45 ms per step in 50 - 90
# us gaps between the first MBConv blocks' kernels; with either the branches or the forks off
# (three or two streams) it did not (scripts/step_timeline.py, profiles/r06/graph_gaps.txt).  The
# camera branch's own work (the depth head, forward and backward) and the forks are at
# different points of the step.
_WGRAD_STREAM = [os.environ.get("E2EP_WGRAD_STREAM", "own")]
# diagnostics only (scripts/diag_branch_capture.py): allow the nested fork from a branch stream
# that made the round-4 capture segfault, to see what graphs.capture's join check reports
_FORK_FROM_BRANCH = os.environ.get("E2EP_FORK_FROM_BRANCH", "0") == "1"


def side_stream(device):
    """The weight-gradient side stream of the current stream (one per stream)."""
    idx = device.index if device.index is not None else torch.cuda.current_device()
    if _WGRAD_STREAM[0] in ("cam", "heads"):
        return streams._side(torch.device("cuda", idx), _WGRAD_STREAM[0])
    key = (idx, torch.cuda.current_stream(idx).cuda_stream)
    st = _SIDE.get(key)
    if st is None:
        st = _SIDE[key] = torch.cuda.Stream(device=idx)
    return st


class _Fork:
    """with _Fork(dev) as side: ...launches on `side`...  — forks from the current stream on
    entry (side waits for it); join() makes the current stream wait for the side stream.
    work_us: the side work's estimate (est_us); below E2EP_FORK_MIN_US it stays serial.

    Never forks from a model-branch side stream (e2ep_amd.streams): a stream forked from a
    stream that is itself forked from the capture origin made hipStreamEndCapture segfault
    when the step was graph-captured (scripts/diag_branch_capture.py: model_cam crashed, the
    same capture with no fork inside the branch — model_cam_nofork — replayed correctly;
    profiles/r05/diag_branch_capture.log).  Inside a branch the weight gradient runs after
    the data gradient on the branch's stream, which still overlaps the main stream."""

    def __init__(self, device, on=True, work_us=float("inf")):
        self.main = torch.cuda.current_stream(device)
        self.on = (on and _OVERLAP[0] and work_us >= _FORK_MIN_US[0]
                   and (_FORK_FROM_BRANCH or not streams.is_branch_stream(self.main)))
        self.side = side_stream(device) if self.on else self.main

    def __enter__(self):
        if self.on:
            self.side.wait_stream(self.main)
            self._ctx = torch.cuda.stream(self.side)
            self._ctx.__enter__()
        return self

    def __exit__(self, *exc):
        if self.on:
            self._ctx.__exit__(*exc)
        return False

    def join(self):
        if self.on:
            self.main.wait_stream(self.side)


# Both gradients of a conv layer in one launch (e2ep_conv_bwd, k_conv_bwd_pair) where the
# geometry allows it (e2ep_conv_bwd_pair_ok): no fork / join, the two GEMMs' blocks still run
# concurrently.  E2EP_CONV_PAIR=0 keeps the forked two-launch backward (A/B).
_CONV_PAIR = [os.environ.get("E2EP_CONV_PAIR", "1") != "0"]


def set_conv_pair(on):
    """Enable / disable the one-launch conv backward (returns the previous setting)."""
    prev = _CONV_PAIR[0]
    _CONV_PAIR[0] = bool(on)
    return prev


def _conv_bwd_pair(gy, x, wt, dims, gc, gskip, wshape):
    """(dx, dw) of a conv through e2ep_conv_bwd; dx as _Conv2d.backward's dgrad path builds it."""
    N, Cin, H, W = dims[:4]
    lib = _lib.load()
    d = _lib.dims(dims)
    dw = torch.empty(wshape, dtype=torch.float32, device=x.device)
    splits = lib.e2ep_conv_wgrad_splits(d)
    wsw = torch.empty(splits * dw.numel(), dtype=torch.float32, device=x.device)
    wsd = _ws(lib.e2ep_conv_dgrad_workspace(d, gc), gy.device)
    res = gskip.contiguous() if (gskip is not None and gc == Cin) else None
    dxg = torch.empty(N, gc, H, W, dtype=x.dtype, device=x.device)  # bf16 for a bf16-stored x
    with timing.region(_rname("conv_bwd", dims, f"gc{gc}"), conv_flops(dims, gc) + conv_flops(dims)):
        _lib.call("e2ep_conv_bwd", _lib.ptr(gy), _lib.ptr(x), _lib.ptr(wt), d, gc, _lib.ptr(res),
                  _lib.ptr(dxg), _lib.ptr(wsd), _lib.nbytes(wsd), splits, _lib.ptr(wsw),
                  _lib.nbytes(wsw), _lib.ptr(dw), _lib.stream(), (_IO_X | _IO_DX) if _io_x(x) else 0)
    if gc == Cin:
        dx = dxg
    elif gskip is not None:  # channels past gc get only the skip gradient
        dx = gskip.clone()
        dx[:, :gc] += dxg
    else:
        dx = torch.zeros_like(x)
        dx[:, :gc] = dxg
    return dx, dw


class _Conv2d(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, w, b, dims, act, grad_channels, skip=False, stats=None):
        x = x.contiguous()
        wt = tap_major(w)  # one small transpose per step for R*S > 1; shared with dgrad
        N, Cin, H, W, Cout, R, S, P, Q = dims[:9]
        y = conv_fwd(x, wt, b, dims, act, torch.empty(N, Cout, P, Q, dtype=torch.float32, device=x.device),
                     w_layout=1, stats=stats)
        ctx.dims, ctx.act, ctx.has_bias, ctx.gc = dims, act, b is not None, grad_channels
        ctx.save_for_backward(x, wt, y if act else None)
        ctx.wshape = w.shape
        ctx.skip = skip
        # an unused skip alias (a trunk endpoint nobody reads) arrives as None, not as a
        # zero-filled gradient
        ctx.set_materialize_grads(False)
        # skip: also hand x back, so the block's skip connection reads it from here and its
        # gradient arrives in this backward, where the data-gradient epilogue adds it
        return (y, x) if skip else y

    @staticmethod
    def backward(ctx, gy, gskip=None):
        x, wt, y = ctx.saved_tensors
        dims = ctx.dims
        N, Cin, H, W, Cout, R, S, P, Q = dims[:9]
        gy = gy.contiguous()
        s = _lib.stream()
        if ctx.act == 1:  # ReLU gradient mask (y > 0 <=> pre-activation > 0), one e2ep launch
            gm = torch.empty_like(gy)
            _lib.call("e2ep_act_bwd", _lib.ptr(y), _lib.ptr(gy), gy.numel(), 1, _lib.ptr(gm), s)
            gy = gm
        dx = dw = db = None
        # weight / bias gradients on the side stream, concurrent with the data gradient
        want_w, want_b = ctx.needs_input_grad[1], ctx.has_bias and ctx.needs_input_grad[2]
        gc = ctx.gc or Cin
        # a bf16-stored x (C3 precision: the pair is then k_lp_bwd_pair) pairs without a skip
        # gradient only
        xb = x.dtype == torch.bfloat16
        if want_w and ctx.needs_input_grad[0] and _CONV_PAIR[0] and (not xb or gskip is None) and \
                _lib.load().e2ep_conv_bwd_pair_ok(_lib.dims(dims), gc):
            dx, dw = _conv_bwd_pair(gy, x, wt, dims, gc, gskip, ctx.wshape)
            if want_b:
                db = torch.empty(Cout, dtype=torch.float32, device=x.device)
                _lib.call("e2ep_bias_grad", _lib.ptr(gy), N, Cout, P * Q, _lib.ptr(db), s)
            return dx, dw, db, None, None, None, None, None
        fork = None
        if want_w or want_b:
            if want_w:  # allocated on the current stream (see _Fork)
                dw = torch.empty(ctx.wshape, dtype=torch.float32, device=x.device)
                ws = torch.empty(_lib.load().e2ep_conv_wgrad_splits(_lib.dims(dims)) * dw.numel(),
                                 dtype=torch.float32, device=x.device)
            if want_b:
                db = torch.empty(Cout, dtype=torch.float32, device=x.device)
            fork = _Fork(x.device, on=ctx.needs_input_grad[0], work_us=est_us(conv_flops(dims)))
            with fork:
                if want_w:
                    conv_wgrad(gy, x, dims, dw, ws)
                if want_b:
                    _lib.call("e2ep_bias_grad", _lib.ptr(gy), N, Cout, P * Q, _lib.ptr(db),
                              _lib.stream())
        if ctx.needs_input_grad[0]:
            res = gskip.contiguous() if (gskip is not None and gc == Cin) else None
            dxg = conv_dgrad(gy, wt, dims, gc, torch.empty(N, gc, H, W, dtype=x.dtype, device=x.device),
                             w_layout=1, res=res)
            if gc == Cin:
                dx = dxg
            elif gskip is not None:  # channels past gc get only the skip gradient
                dx = gskip.clone()
                dx[:, :gc] += dxg
            else:
                dx = torch.zeros_like(x)
                dx[:, :gc] = dxg
        if fork is not None:
            fork.join()
        if dx is None and gskip is not None and ctx.needs_input_grad[0]:
            dx = gskip
        return dx, dw, db, None, None, None, None, None


def _skinny(A, ai, ak, B, bk, bj, bias, Mi, Nj, K, out):
    _lib.call("e2ep_skinny_gemm", _lib.ptr(A), ai, ak, _lib.ptr(B), bk, bj, _lib.ptr(bias), Mi, Nj,
              K, _lib.ptr(out), _lib.stream())
    return out


class _Linear1x1(torch.autograd.Function):
    """1x1 conv on a 1x1 map == linear layer y[n, m] = sum_k W[m, k] x[n, k] + b[m]."""

    @staticmethod
    def forward(ctx, x, w, b):
        N, K = x.shape[0], x.shape[1]
        M = w.shape[0]
        x2 = x.reshape(N, K).contiguous()
        w2 = w.reshape(M, K).contiguous()
        y = torch.empty(N, M, dtype=torch.float32, device=x.device)
        _skinny(x2, K, 1, w2, 1, K, b, N, M, K, y)
        ctx.save_for_backward(x2, w2)
        ctx.has_bias, ctx.wshape, ctx.xshape = b is not None, w.shape, x.shape
        return y.view(N, M, 1, 1)

    @staticmethod
    def backward(ctx, gy):
        x2, w2 = ctx.saved_tensors
        N, K = x2.shape
        M = w2.shape[0]
        g = gy.reshape(N, M).contiguous()
        dx = dw = db = None
        if ctx.needs_input_grad[0]:
            dx = _skinny(g, M, 1, w2, K, 1, None, N, K, M,
                         torch.empty(N, K, dtype=torch.float32, device=g.device)).view(ctx.xshape)
        if ctx.needs_input_grad[1]:
            dw = _skinny(g, 1, M, x2, K, 1, None, M, K, N,
                         torch.empty(M, K, dtype=torch.float32, device=g.device)).view(ctx.wshape)
        if ctx.has_bias and ctx.needs_input_grad[2]:
            db = torch.empty(M, dtype=torch.float32, device=g.device)
            _lib.call("e2ep_bias_grad", _lib.ptr(g), N, M, 1, _lib.ptr(db), _lib.stream())
        return dx, dw, db


def conv2d(x, w, b=None, stride=(1, 1), pad=(0, 0, 0, 0), dilation=(1, 1), act=0, grad_channels=None,
           skip=False, bn_stats=False):
    """pad = (left, right, top, bottom); act 0 none, 1 relu (fused epilogue).
    skip=True returns (y, x_skip): use x_skip for the block's skip connection and its gradient
    is added to this conv's input gradient inside the data-gradient kernel.
    bn_stats=True (a training BatchNorm reads y next): where the routed kernel takes them and
    the BN would make a statistics pass over y (e2ep_bn_fwd_split), the epilogue also writes
    y's per-channel partial sums (e2ep_conv_fwd_stats), attached to y for the BN
    (bn_partials), which then never re-reads y for its statistics."""
    if not x.is_cuda:
        raise _lib.E2EPError("e2ep conv2d runs on a HIP device only")
    N, Cin, H, W = x.shape
    Cout, cin_w, R, S = w.shape
    if cin_w != Cin:
        raise _lib.E2EPError(f"e2ep conv2d: groups must be 1 (w {tuple(w.shape)}, x {tuple(x.shape)})")
    if H == 1 and W == 1 and R == 1 and S == 1 and act == 0 and not any(pad) and grad_channels is None:
        y = _Linear1x1.apply(x, w, b)
        return (y, x) if skip else y
    sh, sw = stride
    dh, dw = dilation
    l, r, t, btm = pad
    P = (H + t + btm - dh * (R - 1) - 1) // sh + 1
    Q = (W + l + r - dw * (S - 1) - 1) // sw + 1
    dims = (N, Cin, H, W, Cout, R, S, P, Q, sh, sw, t, l, dh, dw)
    # only where the BN would otherwise make a statistics pass (its split path)
    lib = _lib.load()
    tiles = (lib.e2ep_conv_fwd_stats_tiles(_lib.dims(dims), 1)
             if bn_stats and _BN_STATS[0] and lib.e2ep_bn_fwd_split(N, Cout, P, Q) else 0)
    if tiles <= 0:
        return _Conv2d.apply(x, w, b, dims, act, grad_channels, bool(skip))
    part = torch.empty(Cout * tiles * 2, dtype=torch.float64, device=x.device)
    out = _Conv2d.apply(x, w, b, dims, act, grad_channels, bool(skip), part)
    y = out[0] if skip else out
    y._e2ep_bn_part = (part, tiles)
    return out
