"""bf16 activation storage (C3, e2ep.h E2EP_IO_*): the MBConv depthwise output, the gradient at
it and the depthwise data gradient stored as bf16.

The kernels widen a bf16 element on load and round on store, with the fp32 arithmetic of the
fp32 path, so the checks are exact: fed the same values (bf16-representable inputs as fp32
tensors), the bf16-storage launch returns bitwise the fp32 launch's outputs — a bf16 output
equal to the fp32 output rounded to nearest-even (torch's .to(torch.bfloat16)), fp32 outputs
and parameter gradients equal.  Where the storage itself rounds an intermediate (the depthwise
data gradient handed to _bn0's backward) the module-level result is held to the bf16 budget.
Reference: efficientnet-pytorch MBConvBlock (_bn0 -> swish -> _depthwise_conv -> _bn1 -> swish ->
SE) via model/cam_encoder.py:69-73; BASELINE configs[2] (C3)."""
import pytest
import torch
from torch import nn

from helpers import rel_l2

pytestmark = pytest.mark.gpu
DEV = "cuda"
BF = torch.bfloat16
IO_X, IO_DY, IO_DX = 1, 2, 4


def _g(seed):
    return torch.Generator().manual_seed(seed)


def _bfvals(t):
    """t rounded to bf16, kept as fp32 (the values a bf16 tensor holds)."""
    return t.to(BF).float()


def _bn(C, g, train=True):
    bn = nn.BatchNorm2d(C, momentum=0.01, eps=1e-3)
    with torch.no_grad():
        bn.weight.copy_(1 + 0.3 * torch.randn(C, generator=g))
        bn.bias.copy_(0.2 * torch.randn(C, generator=g))
        bn.running_mean.copy_(0.1 * torch.randn(C, generator=g))
        bn.running_var.copy_(0.5 + torch.rand(C, generator=g))
    return bn.train(train).to(DEV)


DW_CASES = [(8, 192, 64, 64, 3, 1, (1, 1, 1, 1)), (8, 336, 32, 32, 5, 1, (2, 2, 2, 2)),
            (32, 672, 16, 16, 3, 1, (1, 1, 1, 1)), (4, 144, 64, 64, 3, 2, (0, 1, 0, 1)),
            (4, 192, 32, 32, 5, 2, (2, 2, 2, 2)), (8, 144, 128, 128, 3, 2, (0, 1, 0, 1)),
            (32, 144, 128, 128, 3, 2, (0, 1, 0, 1))]


def _dims(case):
    N, C, H, W, K, s, pad = case
    P, Q = (H + pad[2] + pad[3] - K) // s + 1, (W + pad[0] + pad[1] - K) // s + 1
    return (N, C, H, W, K, P, Q, s, pad[2], pad[0]), P, Q


@pytest.mark.parametrize("case", DW_CASES)
def test_depthwise_bf16_io_bitwise(case):
    """e2ep_dwconv_fwd_stats (y bf16, statistics of the stored values: within fp32
    rounding of the fp64 sums of the bf16 output), e2ep_dwconv_bwd /
    _dgrad / _wgrad (gy and dx bf16) against the fp32 launches on the same values."""
    from e2ep_amd import _lib
    lib = _lib.load()
    N, C, H, W, K, s, pad = case
    dims, P, Q = _dims(case)
    d = _lib.dims(dims)
    g = _g(C + H + K)
    x = (torch.randn(N, C, H, W, generator=g) * 2 + 0.5).to(DEV)
    w = (torch.randn(C, 1, K, K, generator=g) / K).to(DEV)
    sc = (1 + 0.3 * torch.randn(C, generator=g)).to(DEV)
    sh = (0.2 * torch.randn(C, generator=g)).to(DEV)
    gy32 = _bfvals(torch.randn(N, C, P, Q, generator=g)).to(DEV)
    gy16 = gy32.to(BF)
    st = _lib.stream()
    tiles = lib.e2ep_dwconv_fwd_stats_tiles(d)
    assert tiles > 0
    # forward: y bf16 == fp32 y rounded; statistics = fp64 sums of the stored bf16 values
    y32 = torch.empty(N, C, P, Q, device=DEV)
    y16 = torch.empty(N, C, P, Q, device=DEV, dtype=BF)
    s32 = torch.empty(C * tiles * 2, dtype=torch.float64, device=DEV)
    s16 = torch.empty_like(s32)
    for y, stt, io in ((y32, s32, 0), (y16, s16, IO_DX)):
        _lib.call("e2ep_dwconv_fwd_stats", _lib.ptr(x), _lib.ptr(w), d, _lib.ptr(sc), _lib.ptr(sh), 2,
                  _lib.ptr(y), _lib.ptr(stt), _lib.nbytes(stt), st, io)
    assert torch.equal(y16, y32.to(BF))
    part = s16.view(tiles, C, 2).sum(0)
    yv = y16.double()
    # a lane's 4 values are summed in fp32 before the fp64 wave sums (as in the fp32 path)
    assert torch.allclose(part[:, 0], yv.sum((0, 2, 3)), rtol=1e-6, atol=1e-4)
    assert torch.allclose(part[:, 1], (yv * yv).sum((0, 2, 3)), rtol=1e-6, atol=1e-4)
    # backward: paired launch where it exists, and the two separate launches
    ws = torch.empty(max(lib.e2ep_dwconv_wgrad_workspace(d), 16), dtype=torch.uint8, device=DEV)
    outs = {}
    for io, gy, dt in ((0, gy32, torch.float32), (IO_DY | IO_DX, gy16, BF)):
        dx_s, dw_s = torch.empty(N, C, H, W, device=DEV, dtype=dt), torch.empty_like(w)
        _lib.call("e2ep_dwconv_dgrad", _lib.ptr(gy), _lib.ptr(w), d, _lib.ptr(dx_s), st, io)
        _lib.call("e2ep_dwconv_wgrad", _lib.ptr(gy), _lib.ptr(x), d, _lib.ptr(sc), _lib.ptr(sh), 2,
                  _lib.ptr(ws), _lib.nbytes(ws), _lib.ptr(dw_s), st, io & IO_DY)
        outs[io] = [dx_s, dw_s]
        if lib.e2ep_dwconv_bwd_pair_ok(d):
            dx_p, dw_p = torch.empty_like(dx_s), torch.empty_like(w)
            _lib.call("e2ep_dwconv_bwd", _lib.ptr(gy), _lib.ptr(x), _lib.ptr(w), d, _lib.ptr(sc),
                      _lib.ptr(sh), 2, _lib.ptr(dx_p), _lib.ptr(ws), _lib.nbytes(ws), _lib.ptr(dw_p),
                      st, io)
            outs[io] += [dx_p, dw_p]
    f32, b16 = outs[0], outs[IO_DY | IO_DX]
    for i in range(0, len(f32), 2):
        assert torch.equal(b16[i], f32[i].to(BF))  # dx
        assert torch.equal(b16[i + 1], f32[i + 1])  # dw


@pytest.mark.parametrize("shape", [(32, 672, 16, 16), (8, 336, 32, 32), (8, 192, 64, 64),
                                   (32, 144, 64, 64)])
@pytest.mark.parametrize("bn_small", [1, 0], ids=["bn_one_launch", "bn_split"])
def test_bn_bwd_bf16_io_bitwise(shape, bn_small):
    """e2ep_bn_bwd with (x, dx) bf16 and a squeeze-excitation gate (_bn1), with dy bf16 (_bn0),
    e2ep_bn_bwd_planes with (x, dx) bf16 and e2ep_bn_stats with x bf16, against the fp32
    launches on the same values."""
    from e2ep_amd import _lib
    lib = _lib.load()
    prev = _lib.call_raw("e2ep_bn_small", bn_small)
    try:
        N, C, H, W = shape
        g = _g(C + H)
        x32 = _bfvals(torch.randn(N, C, H, W, generator=g) * 2 + 0.5).to(DEV)
        dy32 = _bfvals(torch.randn(N, C, H, W, generator=g)).to(DEV)
        mean = (x32.mean((0, 2, 3)) + 0.01).contiguous()
        invstd = (1 / (x32.var((0, 2, 3)) + 1e-3).sqrt()).contiguous()
        gam = (1 + 0.3 * torch.randn(C, generator=g)).to(DEV)
        bet = (0.2 * torch.randn(C, generator=g)).to(DEV)
        logit = torch.randn(N, C, generator=g).to(DEV)
        dpool = torch.randn(N, C, generator=g).to(DEV)
        ws = torch.empty(max(lib.e2ep_bn_workspace(N, C, H, W), 16), dtype=torch.uint8, device=DEV)
        st = _lib.stream()

        def bwd(x, dy, io, gate, dxdt):
            dx = torch.empty(N, C, H, W, device=DEV, dtype=dxdt)
            dg, db = torch.empty_like(gam), torch.empty_like(bet)
            _lib.call("e2ep_bn_bwd", _lib.ptr(x), _lib.ptr(dy), _lib.ptr(mean), _lib.ptr(invstd),
                      _lib.ptr(gam), _lib.ptr(bet), None, None, 1.0,
                      _lib.ptr(logit) if gate else None, _lib.ptr(dpool) if gate else None,
                      N, C, H, W, 1, 2, _lib.ptr(dx), _lib.ptr(dg), _lib.ptr(db), None, _lib.ptr(ws),
                      _lib.nbytes(ws), st, io)
            return dx, dg, db

        # _bn1: x and dx bf16, gated
        a = bwd(x32, dy32, 0, True, torch.float32)
        b = bwd(x32.to(BF), dy32, IO_X | IO_DX, True, BF)
        assert torch.equal(b[0], a[0].to(BF)) and torch.equal(b[1], a[1]) and torch.equal(b[2], a[2])
        # _bn1 behind a bf16-stored squeeze-excitation output: x, dy and dx bf16, gated
        b = bwd(x32.to(BF), dy32.to(BF), IO_X | IO_DY | IO_DX, True, BF)
        assert torch.equal(b[0], a[0].to(BF)) and torch.equal(b[1], a[1]) and torch.equal(b[2], a[2])
        # _bn0: dy bf16
        a = bwd(x32, dy32, 0, False, torch.float32)
        b = bwd(x32, dy32.to(BF), IO_DY, False, torch.float32)
        assert all(torch.equal(u, v) for u, v in zip(a, b))
        # statistics of a bf16 x
        outs = []
        for x, io in ((x32, 0), (x32.to(BF), IO_X)):
            o = torch.empty(4, C, device=DEV)
            _lib.call("e2ep_bn_stats", _lib.ptr(x), _lib.ptr(gam), _lib.ptr(bet), None, None, N, C, H, W,
                      1, 0.01, 1e-3, _lib.ptr(o[0]), _lib.ptr(o[1]), _lib.ptr(o[2]), _lib.ptr(o[3]),
                      _lib.ptr(ws), _lib.nbytes(ws), st, io)
            outs.append(o)
        assert torch.equal(outs[0], outs[1])
        # the apply pass from per-plane sums (split BN only)
        planes = torch.randn(N * C * 4, generator=g, dtype=torch.float64).to(DEV)
        res = []
        for x, io, dt in ((x32, 0, torch.float32), (x32.to(BF), IO_X | IO_DX, BF)):
            dx = torch.empty(N, C, H, W, device=DEV, dtype=dt)
            dg, db = torch.empty_like(gam), torch.empty_like(bet)
            _lib.call("e2ep_bn_bwd_planes", _lib.ptr(x), _lib.ptr(dy32), _lib.ptr(mean), _lib.ptr(invstd),
                      _lib.ptr(gam), _lib.ptr(bet), _lib.ptr(logit), _lib.ptr(dpool), _lib.ptr(planes),
                      N, C, H, W, 2, _lib.ptr(dx), _lib.ptr(dg), _lib.ptr(db), st, io)
            res.append((dx, dg, db))
        assert torch.equal(res[1][0], res[0][0].to(BF))
        assert torch.equal(res[1][1], res[0][1]) and torch.equal(res[1][2], res[0][2])
        # masks the kernels were not built for are refused
        assert lib.e2ep_bn_bwd(_lib.ptr(x32), _lib.ptr(dy32), _lib.ptr(mean), _lib.ptr(invstd), None,
                               None, None, None, 1.0, None, None, N, C, H, W, 1, 2, _lib.ptr(ws),
                               None, None, None, _lib.ptr(ws), _lib.nbytes(ws), st, IO_X) != 0
    finally:
        _lib.call_raw("e2ep_bn_small", prev)


@pytest.mark.parametrize("case", [(32, 672, 16, 16, 28), (8, 336, 32, 32, 14), (8, 192, 64, 64, 8),
                                  (6, 56, 30, 30, 14)])
def test_squeeze_excite_bf16_input_bitwise(case):
    """The fused _bn1 -> swish -> SE op fed a bf16 x (nn_ops.bn_swish_squeeze_excite dispatches
    on its dtype; its output is then stored bf16 as well) against the same op fed the same
    values in fp32: output (rounded) and every gradient bitwise (the input gradient bf16 = the
    fp32 one rounded), with and without the SE-pass BN sums."""
    from e2ep_amd import nn_ops
    N, C, H, W, sq = case
    lv = nn_ops.set_bf16_store(2)  # the output stored bf16 as well
    for sums in (True, False):
        prev = nn_ops.set_se_bn_sums(sums)
        try:
            g = _g(C + sq + H)
            x = _bfvals(torch.randn(N, C, H, W, generator=g) * 2 + 0.5)
            w1 = torch.randn(sq, C, 1, 1, generator=g) / C ** 0.5
            b1 = torch.randn(sq, generator=g) * 0.1
            w2 = torch.randn(C, sq, 1, 1, generator=g) / sq ** 0.5
            b2 = torch.randn(C, generator=g) * 0.1
            dy = _bfvals(torch.randn(N, C, H, W, generator=g)).to(DEV)
            res = []
            for dt in (torch.float32, BF):
                bn = _bn(C, _g(C))
                ts = [x.to(DEV).to(dt).requires_grad_(True)] + \
                     [t.to(DEV).requires_grad_(True) for t in (w1, b1, w2, b2)]
                y = nn_ops.bn_swish_squeeze_excite(ts[0], bn, *ts[1:])
                y.backward(dy.to(y.dtype))
                res.append((y.detach(), [t.grad for t in ts], bn.weight.grad, bn.bias.grad,
                            bn.running_mean.clone(), bn.running_var.clone()))
            (y0, g0, gw0, gb0, rm0, rv0), (y1, g1, gw1, gb1, rm1, rv1) = res
            assert y1.dtype == BF and torch.equal(y1, y0.to(BF))
            assert g1[0].dtype == BF and torch.equal(g1[0], g0[0].to(BF))
            assert all(torch.equal(a, b) for a, b in zip(g1[1:], g0[1:]))
            assert torch.equal(gw1, gw0) and torch.equal(gb1, gb0)
            assert torch.equal(rm1, rm0) and torch.equal(rv1, rv0)
        finally:
            nn_ops.set_se_bn_sums(prev)
    nn_ops.set_bf16_store(lv)


# (N, Cin, H, W, Cout): MBConv project convs (1x1); Cout 32 runs k_conv_gemm forward and data
# gradient (M or K of 32), the others k_conv_lp / k_lp_bwd_pair; the weight gradient k_wgrad_lp
PROJ_CASES = [(32, 672, 16, 16, 112), (16, 336, 32, 32, 56), (8, 192, 64, 64, 32),
              (32, 960, 16, 16, 160)]


@pytest.mark.parametrize("case", PROJ_CASES)
@pytest.mark.parametrize("pair", [True, False], ids=["pair", "two_launches"])
def test_project_conv_bf16_input_bitwise(case, pair):
    """C3 precision: a 1x1 conv fed a bf16 x (the bf16-stored SE output) against the same conv
    fed the same values in fp32 — output, weight gradient bitwise; the data gradient bf16 = the
    fp32 one rounded — paired backward and two launches."""
    from e2ep_amd import conv, ops, precision
    N, Cin, H, W, Cout = case
    g = _g(Cin + Cout + H)
    x = _bfvals(torch.randn(N, Cin, H, W, generator=g)).to(DEV)
    w = (torch.randn(Cout, Cin, 1, 1, generator=g) / Cin ** 0.5).to(DEV)
    gy = torch.randn(N, Cout, H, W, generator=g).to(DEV)
    res = []
    prev = conv.set_conv_pair(pair)
    try:
        with precision.use("bf16"):
            for dt in (torch.float32, BF):
                xd = x.to(dt).clone().requires_grad_(True)
                wd = w.clone().requires_grad_(True)
                y = ops.conv2d(xd, wd, None, 1, (0, 0, 0, 0))
                y.backward(gy)
                res.append((y.detach(), xd.grad, wd.grad))
    finally:
        conv.set_conv_pair(prev)
    (y0, dx0, dw0), (y1, dx1, dw1) = res
    assert y1.dtype == torch.float32 and torch.equal(y1, y0)
    assert dx1.dtype == BF and torch.equal(dx1, dx0.to(BF))
    assert torch.equal(dw1, dw0)


@pytest.mark.parametrize("case", DW_CASES[:6])
def test_bn_swish_depthwise_bf16_store(case):
    """nn_ops.bn_act_depthwise_conv2d in a bf16-precision training forward stores its output
    bf16 (E2EP_BF16_STORE): the output is the fp32-storage output rounded, the weight gradient
    is bitwise the fp32-storage one (same gy values), and the input / BN-parameter gradients —
    which pass through the bf16-stored depthwise data gradient — stay within the bf16 budget
    (rel-L2 <= 8e-3) of the fp32-storage step."""
    from e2ep_amd import nn_ops, precision
    N, C, H, W, K, s, pad = case
    g = _g(C + H + K + 1)
    x = torch.randn(N, C, H, W, generator=g) * 2 + 0.5
    w = torch.randn(C, 1, K, K, generator=g) / K
    res = {}
    with precision.use("bf16"):
        for store in (False, True):
            prev = nn_ops.set_bf16_store(store)
            try:
                bn = _bn(C, _g(C + 7))
                xd = x.to(DEV).requires_grad_(True)
                wd = w.to(DEV).requires_grad_(True)
                y = nn_ops.bn_act_depthwise_conv2d(xd, bn, "swish", wd, s, pad, bn_stats=True)
                gy = _bfvals(torch.randn(y.shape, generator=_g(5))).to(DEV).to(y.dtype)
                y.backward(gy)
                res[store] = (y.detach(), xd.grad, wd.grad, bn.weight.grad, bn.bias.grad)
            finally:
                nn_ops.set_bf16_store(prev)
    (y0, dx0, dw0, dg0, db0), (y1, dx1, dw1, dg1, db1) = res[False], res[True]
    assert y0.dtype == torch.float32 and y1.dtype == BF
    assert torch.equal(y1, y0.to(BF))
    assert torch.equal(dw1, dw0)
    assert dx1.dtype == torch.float32
    assert rel_l2(dx1, dx0) < 8e-3
    assert rel_l2(dg1, dg0) < 8e-3 and rel_l2(db1, db0) < 8e-3


def test_bf16_store_only_in_bf16_training():
    """The storage switch acts in bf16-precision training forwards only: fp32 precision and
    inference forwards keep fp32 depthwise outputs."""
    from e2ep_amd import nn_ops, precision
    C = 32
    x = torch.randn(2, C, 16, 16, device=DEV)
    w = torch.randn(C, 1, 3, 3, device=DEV)
    bn = _bn(C, _g(3))
    prev = nn_ops.set_bf16_store(1)
    try:
        assert nn_ops.bn_act_depthwise_conv2d(x, bn, "swish", w, 1, (1, 1, 1, 1)).dtype == torch.float32
        with precision.use("bf16"):
            assert nn_ops.bn_act_depthwise_conv2d(x, bn, "swish", w, 1, (1, 1, 1, 1)).dtype == BF
            nn_ops.set_bf16_store(0)  # the default: fp32 storage
            assert nn_ops.bn_act_depthwise_conv2d(x, bn, "swish", w, 1, (1, 1, 1, 1)).dtype == torch.float32
            nn_ops.set_bf16_store(1)
            bn.eval()
            with torch.no_grad():
                assert nn_ops.bn_act_depthwise_conv2d(x, bn, "swish", w, 1, (1, 1, 1, 1)).dtype == torch.float32
    finally:
        nn_ops.set_bf16_store(prev)


@pytest.mark.parametrize("case", [(2, 32, 30, 30, 3, 1, (1, 1, 1, 1)),   # W % 4 != 0
                                  (2, 32, 18, 18, 5, 2, (2, 2, 2, 2)),   # stride-2 output 9x9
                                  (2, 16, 20, 20, 3, 2, (1, 1, 1, 1))])  # 10x10 output: no strip kernel
def test_bf16_store_non_strip_geometry_keeps_fp32(case):
    """A layer whose geometry some kernel beside it cannot store in bf16 (no strip kernel,
    P*Q % 4 != 0, ...) keeps fp32 storage under E2EP_BF16_STORE (e2ep_dwconv_bf16_ok, ADVICE
    r5) instead of raising E2EP_EINVAL partway through the step; forward and backward run and
    equal the fp32-storage step bitwise."""
    from e2ep_amd import _lib, nn_ops, precision
    N, C, H, W, K, s, pad = case
    dims, P, Q = _dims(case)
    assert _lib.call_raw("e2ep_dwconv_bf16_ok", _lib.dims(dims)) == 0
    g = _g(C + H + K)
    x = torch.randn(N, C, H, W, generator=g)
    w = torch.randn(C, 1, K, K, generator=g) / K
    res = {}
    with precision.use("bf16"):
        for store in (0, 2):
            prev = nn_ops.set_bf16_store(store)
            try:
                bn = _bn(C, _g(C + 7))
                xd = x.to(DEV).requires_grad_(True)
                wd = w.to(DEV).requires_grad_(True)
                y = nn_ops.bn_act_depthwise_conv2d(xd, bn, "swish", wd, s, pad)
                y.backward(torch.ones_like(y))
                res[store] = (y.detach(), xd.grad, wd.grad)
            finally:
                nn_ops.set_bf16_store(prev)
    assert res[2][0].dtype == torch.float32
    for a, b in zip(res[0], res[2]):
        assert torch.equal(a, b)
