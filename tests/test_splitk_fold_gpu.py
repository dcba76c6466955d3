"""Split-K reductions folded into their producing launch (e2ep_tune key 28 = 2, the default):
the last-arriving split of an output tile sums every split's slab in split order and writes
the final values (bias, ReLU, residual gradient, row sums) — csrc/handoff.h, the write-through
(sc1) hand-off of cdna_hip_programming.md §6 Guideline 16.

The fold keeps the separate reduction kernels' summation order, so for every kernel family
(k_conv_gemm, k_conv_lp fp32 / bf16, k_gemm incl. the row-sum column) the folded result must
equal the two-launch result BIT FOR BIT, run after run, and both match fp64 within the fp32
bound.  Each case runs back to back several times with other work in flight on a second
stream (uneven load), so tiles' splits land on different XCDs and arrive in varying order."""
import pytest
import torch
import torch.nn.functional as F

from helpers import rel_l2

pytestmark = pytest.mark.gpu
DEV = "cuda"


def _tune(key, value):
    from e2ep_amd import _lib
    return _lib.load().e2ep_tune(key, value)


class _Tunes:
    def __init__(self, **kv):
        self.kv = kv

    def __enter__(self):
        self.prev = {k: _tune(int(k[1:]), v) for k, v in self.kv.items()}

    def __exit__(self, *a):
        for k, v in self.prev.items():
            _tune(int(k[1:]), v)


def _noise_stream():
    """Keep the chip unevenly busy while the folded launches run (a long streaming copy on a
    side stream)."""
    s = torch.cuda.Stream()
    big = torch.empty(64 << 20, device=DEV)
    with torch.cuda.stream(s):
        for _ in range(4):
            big.mul_(1.0001)
    return s


# (N, Cin, H, W, Cout, R, S, stride, pad, bias, act): small grids, so the plans split K
CONV = [(2, 160, 8, 8, 960, 1, 1, 1, 0, False, 0), (4, 320, 16, 16, 64, 1, 1, 1, 0, True, 1),
        (2, 64, 16, 16, 64, 3, 3, 1, 1, False, 1), (2, 256, 8, 8, 256, 3, 3, 1, 1, True, 0),
        (3, 100, 8, 8, 70, 1, 1, 1, 0, True, 0), (1, 216, 12, 12, 48, 3, 3, 1, 1, False, 0)]


def _conv_once(case, x, w, b, gy, res):
    from e2ep_amd import conv
    N, Cin, H, W, Cout, R, S, st, p, bias, act = case
    P = (H + 2 * p - R) // st + 1
    Q = (W + 2 * p - S) // st + 1
    dims = (N, Cin, H, W, Cout, R, S, P, Q, st, st, p, p, 1, 1)
    wt = conv.tap_major(w)
    y = conv.conv_fwd(x, wt, b, dims, act, torch.empty(N, Cout, P, Q, device=DEV), w_layout=1)
    dx = conv.conv_dgrad(gy, wt, dims, Cin, torch.empty(N, Cin, H, W, device=DEV), w_layout=1,
                         res=res)
    return y, dx


@pytest.mark.parametrize("case", CONV, ids=[str(i) for i in range(len(CONV))])
@pytest.mark.parametrize("family", ["conv_gemm", "conv_lp_fp32", "conv_lp_bf16"])
def test_conv_split_fold_bitwise_equals_two_launch(case, family):
    from e2ep_amd import precision
    N, Cin, H, W, Cout, R, S, st, p, bias, act = case
    g = torch.Generator().manual_seed(N * 31 + Cin + Cout)
    x = torch.randn(N, Cin, H, W, generator=g)
    w = torch.randn(Cout, Cin, R, S, generator=g) / (Cin * R * S) ** 0.5
    b = torch.randn(Cout, generator=g) if bias else None
    P = (H + 2 * p - R) // st + 1
    gy = torch.randn(N, Cout, P, P, generator=g)
    res = torch.randn(N, Cin, H, W, generator=g)
    dev = [t.to(DEV) if t is not None else None for t in (x, w, b, gy, res)]
    # k_conv_gemm everywhere, 4 forced splits (key 8 = splits + 1); k_conv_lp: every shape on
    # the lp kernel (key 10 forces a tile, key 14 the fp32 variant), its automatic split plan
    kv = {"conv_gemm": dict(k8=5, k14=1, k11=1), "conv_lp_fp32": dict(k10=11, k14=2),
          "conv_lp_bf16": dict(k10=11)}[family]
    prec = "bf16" if family == "conv_lp_bf16" else "fp32"
    from e2ep_amd import _lib
    old_var = _lib.call_raw("e2ep_conv_gemm_variant", 1 if family == "conv_gemm" else 0)
    try:
        with precision.use(prec), _Tunes(**kv):
            with _Tunes(k28=1):
                y1, d1 = _conv_once(case, *dev)
            outs = []
            for _ in range(3):
                s = _noise_stream()
                with _Tunes(k28=2):
                    outs.append(_conv_once(case, *dev))
                torch.cuda.current_stream().wait_stream(s)
            torch.cuda.synchronize()
    finally:
        _lib.call_raw("e2ep_conv_gemm_variant", old_var)
    for y2, d2 in outs:
        assert torch.equal(y1, y2), family
        assert torch.equal(d1, d2), family
    if family != "conv_lp_bf16":
        y64 = F.conv2d(x.double(), w.double(), b.double() if bias else None, st, p)
        if act:
            y64 = y64.clamp_min(0)
        d64 = torch.nn.grad.conv2d_input(x.shape, w.double(), gy.double(), st, p) + res.double()
        assert rel_l2(y1, y64) < 2e-6 and rel_l2(d1, d64) < 2e-6


@pytest.mark.parametrize("tile", [1, 2, 3, 4, 5, 6])
@pytest.mark.parametrize("splits", [2, 3, 8])
def test_gemm_split_fold_bitwise_equals_two_launch(tile, splits):
    """k_gemm at every tile with K split 2 / 3 / 8: plain, bias + residual + ReLU, and the
    row-sum (bias-gradient) column: folded == two-launch, bitwise, under uneven load."""
    from e2ep_amd import _lib, nn_ops
    M, N, K = 197, 301, 777
    g = torch.Generator().manual_seed(tile * 10 + splits)
    A = torch.randn(M, K, generator=g).to(DEV)
    B = torch.randn(N, K, generator=g).to(DEV)
    bias, cadd = torch.randn(N, generator=g).to(DEV), torch.randn(M, N, generator=g).to(DEV)
    rows = torch.randn(K, M, generator=g).to(DEV)

    def run():
        a = nn_ops.gemm(A, True, B, True, M, N, K)
        c = nn_ops.gemm(A, True, B, True, M, N, K, bias=bias, cadd=cadd, relu=True)
        dw = torch.empty(M, N, device=DEV)
        db = torch.empty(M, device=DEV)
        nb = _lib.load().e2ep_gemm_rowsum_workspace(M, N, K)
        ws = torch.empty(max(1, nb // 4), device=DEV)
        bt = B.t().contiguous()
        _lib.call("e2ep_gemm_rowsum", _lib.ptr(rows), rows.stride(0), _lib.ptr(bt), bt.stride(0),
                  _lib.ptr(dw), N, _lib.ptr(db), M, N, K, _lib.ptr(ws), _lib.nbytes(ws), _lib.stream())
        return a, c, dw, db

    try:
        _lib.call("e2ep_gemm_force", tile, splits, 0)
        with _Tunes(k28=1):
            ref = run()
        for _ in range(3):
            s = _noise_stream()
            with _Tunes(k28=2):
                got = run()
            torch.cuda.current_stream().wait_stream(s)
            for a, b in zip(ref, got):
                assert torch.equal(a, b), (tile, splits)
    finally:
        _lib.call("e2ep_gemm_force", 0, 0, 0)
    want = A.double() @ B.double().t()
    assert rel_l2(ref[0], want) < 2e-6
    assert rel_l2(ref[2], rows.double().t() @ B.double().t()) < 2e-6
    assert rel_l2(ref[3], rows.double().sum(0)) < 2e-6


@pytest.mark.parametrize("case", [(4, 144, 64, 64, 3, 2, (0, 1, 0, 1)), (2, 672, 16, 16, 5, 1, (2, 2, 2, 2)),
                                  (2, 24, 128, 128, 3, 1, (1, 1, 1, 1)), (3, 8, 13, 11, 3, 2, (0, 1, 0, 1)),
                                  (32, 960, 16, 16, 5, 1, (2, 2, 2, 2)), (32, 144, 128, 128, 3, 2, (0, 1, 0, 1))])
def test_depthwise_wgrad_fold_bitwise_equals_finalize(case):
    """Depthwise weight gradient: per-channel split slabs summed by the channel's last-arriving
    split (or written directly with one split) == the k_dw_wgrad_finalize launch, bitwise,
    under uneven load; and vs fp64."""
    from e2ep_amd import ops
    N, C, H, W, K, st, pad = case
    g = torch.Generator().manual_seed(C + H + K)
    x = torch.randn(N, C, H, W, generator=g)
    w = torch.randn(C, 1, K, K, generator=g) / K
    xd = x.to(DEV)
    y = ops.conv2d(xd, w.to(DEV), None, st, pad, 1, groups=C)
    dy = torch.randn(y.shape, generator=g).to(DEV)

    def wgrad():
        wd = w.to(DEV).requires_grad_(True)
        ops.conv2d(xd, wd, None, st, pad, 1, groups=C).backward(dy)
        return wd.grad

    with _Tunes(k28=1):
        ref = wgrad()
    for _ in range(3):
        s = _noise_stream()
        with _Tunes(k28=2):
            got = wgrad()
        torch.cuda.current_stream().wait_stream(s)
        assert torch.equal(ref, got)
    w64 = w.double().requires_grad_(True)
    F.conv2d(F.pad(x.double(), pad), w64, None, st, 0, 1, C).backward(dy.double().cpu())
    assert rel_l2(ref, w64.grad) < 2e-5
