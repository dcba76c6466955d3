"""BatchNorm statistics from the producing conv's epilogue (e2ep_conv_fwd_stats ->
e2ep_bn_finalize_part -> e2ep_bn_apply / the depthwise kernel's on-load BN).

The conv output must be bit-identical to e2ep_conv_fwd (the statistics only read the stored
values), the partial sums must match fp64 sums of that output per channel, run after run
bitwise, for every k_conv_gemm tile (64 / 32-row blocks, 64 / 128 / 256-column tiles), with
and without the in-launch split-K fold; and a training BatchNorm fed the partials must match
the same BatchNorm computing its own statistics (forward, running stats, backward)."""
import pytest
import torch
import torch.nn.functional as F

from helpers import rel_l2

pytestmark = pytest.mark.gpu
DEV = "cuda"


def _tune(key, value):
    from e2ep_amd import _lib
    return _lib.load().e2ep_tune(key, value)


# (N, Cin, H, W, Cout, R, S, stride, pad): MBConv expand / project 1x1s at the C2 shapes'
# channel counts (reduced N), a ragged Cout, a 3x3, a map whose pixel count is not a tile
# multiple
CASES = [(4, 24, 32, 32, 144, 1, 1, 1, 0), (4, 144, 32, 32, 32, 1, 1, 1, 0),
         (2, 56, 16, 16, 336, 1, 1, 1, 0), (3, 100, 9, 7, 70, 1, 1, 1, 0),
         (2, 40, 16, 16, 48, 3, 3, 1, 1), (2, 672, 16, 16, 160, 1, 1, 1, 0),
         (5, 24, 13, 11, 24, 1, 1, 1, 0)]


def _dims(case):
    N, Cin, H, W, Cout, R, S, st, p = case
    P = (H + 2 * p - R) // st + 1
    Q = (W + 2 * p - S) // st + 1
    return (N, Cin, H, W, Cout, R, S, P, Q, st, st, p, p, 1, 1)


def _run(case, x, wt, splits_key=None):
    from e2ep_amd import _lib, conv
    d = _dims(case)
    N, Cout, P, Q = d[0], d[4], d[7], d[8]
    tiles = _lib.load().e2ep_conv_fwd_stats_tiles(_lib.dims(d), 1)
    if tiles <= 0:
        return None
    y0 = conv.conv_fwd(x, wt, None, d, 0, torch.empty(N, Cout, P, Q, device=DEV), w_layout=1)
    part = torch.full((Cout * tiles * 2,), float("nan"), dtype=torch.float64, device=DEV)
    y = conv.conv_fwd(x, wt, None, d, 0, torch.empty(N, Cout, P, Q, device=DEV), w_layout=1,
                      stats=part)
    return y0, y, part.view(tiles, Cout, 2), tiles  # tile-major (bnstats.h)


@pytest.mark.parametrize("case", CASES, ids=[str(i) for i in range(len(CASES))])
@pytest.mark.parametrize("plan", ["auto", "split4_fold", "tile32", "lp_bf16", "lp_fp32"])
def test_conv_fwd_stats_partials(case, plan):
    """k_conv_gemm (auto / 4 folded splits / 32-row tiles) and k_conv_lp (bf16 operands, C3;
    the fp32 lp tile on the 3x3)."""
    from e2ep_amd import _lib, conv, precision
    g = torch.Generator().manual_seed(sum(case))
    N, Cin, H, W, Cout, R, S, st, p = case
    x = (torch.randn(N, Cin, H, W, generator=g) + 0.5).to(DEV)
    w = (torch.randn(Cout, Cin, R, S, generator=g) / (Cin * R * S) ** 0.5).to(DEV)
    wt = conv.tap_major(w)
    # split4_fold: 4 K splits folded in-launch (key 8 = splits + 1, key 28 = 2); tile32: the
    # 32-row block tile (key 7 = bm * 1000 + bnt)
    kv = {"auto": {}, "split4_fold": {8: 5, 28: 2}, "tile32": {7: 32128}, "lp_bf16": {},
          "lp_fp32": {14: 2}}[plan]
    prev = {k: _tune(k, v) for k, v in kv.items()}
    old_var = _lib.call_raw("e2ep_conv_gemm_variant", 1)  # k_conv_gemm (the stats kernel)
    try:
        with precision.use("bf16" if plan == "lp_bf16" else "fp32"):
            outs = [_run(case, x, wt) for _ in range(3)]
    finally:
        _lib.call_raw("e2ep_conv_gemm_variant", old_var)
        for k, v in prev.items():
            _tune(k, v)
    if outs[0] is None:
        pytest.skip("routed kernel takes no statistics")
    y0, y, part, tiles = outs[0]
    assert torch.equal(y0, y)  # the statistics do not change the output
    for o in outs[1:]:
        assert torch.equal(o[2], part)  # deterministic
    yd = y.double()
    s_ref = yd.sum(dim=(0, 2, 3))
    q_ref = (yd * yd).sum(dim=(0, 2, 3))
    s, q = part.sum(0).unbind(-1)
    assert torch.isfinite(part).all()
    # a lane's <= 4 values per row summed in fp32 (one rounding of ~6e-8 each), fp64 from the
    # cross-lane reduction on
    assert torch.allclose(s, s_ref, rtol=2e-7, atol=2e-7 * yd.abs().sum().item() / Cout)
    assert torch.allclose(q, q_ref, rtol=2e-7, atol=0)


def test_stats_tiles_zero_where_the_kernel_takes_none():
    """The direct stem conv (Cin*R*S <= 32) takes no statistics: tiles 0, and a stats buffer
    is refused."""
    from e2ep_amd import _lib
    d = (2, 3, 32, 32, 48, 3, 3, 16, 16, 2, 2, 0, 0, 1, 1)
    assert _lib.load().e2ep_conv_fwd_stats_tiles(_lib.dims(d), 1) == 0
    x = torch.randn(2, 3, 32, 32, device=DEV)
    w = torch.randn(9, 48, 3, device=DEV)
    y = torch.empty(2, 48, 16, 16, device=DEV)
    st = torch.empty(4096, dtype=torch.float64, device=DEV)
    with pytest.raises(_lib.E2EPError):
        _lib.call("e2ep_conv_fwd_stats", _lib.ptr(x), _lib.ptr(w), None, _lib.dims(d), 0, 1,
                  _lib.ptr(y), None, 0, _lib.ptr(st), _lib.nbytes(st), _lib.stream(), 0)


@pytest.mark.parametrize("fused", ["bn_act", "bn_act_res_dc", "bn_act_depthwise"])
def test_batchnorm_from_conv_partials_matches_own_statistics(fused):
    """conv2d(bn_stats=True) -> BN: forward, running stats and every gradient agree with the
    same BN computing its own statistics (fp64 sums in another order: within 1e-6), and the
    partial path is taken (the partials are attached to the conv output)."""
    from e2ep_amd import conv, nn_ops
    torch.manual_seed(7)
    N, Cin, H, W, Cout = 16, 32, 32, 32, 192  # N*H*W > 8192: the BN's split path
    x0 = torch.randn(N, Cin, H, W, device=DEV)
    w0 = torch.randn(Cout, Cin, 1, 1, device=DEV) / Cin ** 0.5
    res0 = torch.randn(N, Cout, H, W, device=DEV)
    dc = torch.rand(N, device=DEV)
    wdw = torch.randn(Cout, 1, 3, 3, device=DEV) / 3
    gamma = torch.rand(Cout, device=DEV) + 0.5
    beta = torch.rand(Cout, device=DEV) - 0.5
    results = []
    for use in (False, True):
        bn = torch.nn.BatchNorm2d(Cout, momentum=0.01, eps=1e-3).to(DEV)
        with torch.no_grad():
            bn.weight.copy_(gamma)
            bn.bias.copy_(beta)
        x = x0.clone().requires_grad_(True)
        w = w0.clone().requires_grad_(True)
        y = conv.conv2d(x, w, bn_stats=use)
        assert (conv.bn_partials(y) is not None) == use
        if fused == "bn_act":
            out = nn_ops.batch_norm_act(y, bn, "swish")
        elif fused == "bn_act_res_dc":
            out = nn_ops.batch_norm_act(y, bn, None, res=res0, dc_rand=dc, dc_keep=0.8)
        else:
            out = nn_ops.bn_act_depthwise_conv2d(y, bn, "swish", wdw, 1, (1, 1, 1, 1))
        g = torch.randn(out.shape, generator=torch.Generator().manual_seed(3)).to(DEV)
        out.backward(g)
        results.append((out.detach(), bn.running_mean.clone(), bn.running_var.clone(),
                        x.grad, w.grad, bn.weight.grad, bn.bias.grad))
    for a, b in zip(*results):
        assert rel_l2(b, a.double()) < 1e-6


def test_no_partials_where_the_bn_runs_single_launch():
    """Channels of N*H*W <= 8192 run the single-launch BN (statistics and normalisation from
    registers): no partials are made for them (e2ep_bn_fwd_split = 0)."""
    from e2ep_amd import _lib, conv, nn_ops
    assert _lib.load().e2ep_bn_fwd_split(32, 672, 16, 16) == 0
    assert _lib.load().e2ep_bn_fwd_split(32, 144, 32, 32) == 1
    x = torch.randn(8, 24, 16, 16, device=DEV)
    y = conv.conv2d(x, torch.randn(144, 24, 1, 1, device=DEV), bn_stats=True)
    assert conv.bn_partials(y) is None
    yd = nn_ops.depthwise_conv2d(y, torch.randn(144, 1, 3, 3, device=DEV), 1, (1, 1, 1, 1), bn_stats=True)
    assert conv.bn_partials(yd) is None


def test_batchnorm_partials_ignored_in_eval():
    """An eval-mode BN uses its running statistics, never the conv's batch partials."""
    from e2ep_amd import conv, nn_ops
    torch.manual_seed(9)
    x = torch.randn(2, 24, 16, 16, device=DEV)
    w = torch.randn(144, 24, 1, 1, device=DEV) / 24 ** 0.5
    bn = torch.nn.BatchNorm2d(144).to(DEV).eval()
    with torch.no_grad():
        bn.running_mean.uniform_(-1, 1)
        bn.running_var.uniform_(0.5, 2)
        y = conv.conv2d(x, w, bn_stats=True)
        out = nn_ops.batch_norm_act(y, bn, None)
        ref = F.batch_norm(y.double(), bn.running_mean.double(), bn.running_var.double(),
                           bn.weight.double(), bn.bias.double(), False, 0.0, bn.eps)
    assert rel_l2(out, ref) < 1e-6


# (N, C, H, W, K, stride, pad l r t b): MBConv depthwise shapes (reduced N), ragged row blocks
# (N * P * Q > 8192, so the following BN takes its split path and the partials are made)
DW = [(12, 144, 64, 64, 3, 2, (0, 1, 0, 1)), (40, 672, 16, 16, 5, 1, (2, 2, 2, 2)),
      (9, 192, 32, 32, 5, 1, (2, 2, 2, 2)), (16, 240, 24, 24, 3, 1, (1, 1, 1, 1))]


@pytest.mark.parametrize("case", DW, ids=[str(i) for i in range(len(DW))])
@pytest.mark.parametrize("with_bn0", [False, True])
def test_depthwise_fwd_stats_partials(case, with_bn0):
    """e2ep_dwconv_fwd_stats: y bit-identical to e2ep_dwconv_fwd; per-channel partials sum to
    the fp64 sums of y; bitwise repeatable (the on-load BN0 + swish variant too)."""
    from e2ep_amd import nn_ops
    N, C, H, W, K, st, pad = case
    g = torch.Generator().manual_seed(C + K)
    x = (torch.randn(N, C, H, W, generator=g) + 0.3).to(DEV)
    w = (torch.randn(C, 1, K, K, generator=g) / K).to(DEV)
    bn = torch.nn.BatchNorm2d(C, momentum=0.01, eps=1e-3).to(DEV)

    def run(stats):
        if with_bn0:
            return nn_ops.bn_act_depthwise_conv2d(x, bn, "swish", w, st, pad, bn_stats=stats)
        return nn_ops.depthwise_conv2d(x, w, st, pad, bn_stats=stats)

    y0 = run(False)
    outs = [run(True) for _ in range(2)]
    from e2ep_amd import conv
    pp = conv.bn_partials(outs[0])
    assert pp is not None
    part, tiles = pp
    assert torch.equal(outs[0], y0) and torch.equal(outs[1], y0)
    assert torch.equal(conv.bn_partials(outs[1])[0], part)
    p = part.view(tiles, C, 2).sum(0)
    yd = y0.double()
    assert torch.allclose(p[:, 0], yd.sum(dim=(0, 2, 3)), rtol=2e-7, atol=2e-7 * yd.abs().sum().item() / C)
    assert torch.allclose(p[:, 1], (yd * yd).sum(dim=(0, 2, 3)), rtol=2e-7, atol=0)


def test_bn_swish_se_from_depthwise_partials_matches_own_statistics():
    """depthwise(bn_stats=True) -> _bn1 + swish + SE: forward, running stats and gradients
    agree with the same op computing its own statistics."""
    from e2ep_amd import conv, nn_ops
    torch.manual_seed(11)
    N, C, H, W, sq = 12, 144, 32, 32, 6
    x0 = torch.randn(N, C, H, W, device=DEV)
    wd = torch.randn(C, 1, 3, 3, device=DEV) / 3
    w1, b1 = torch.randn(sq, C, 1, 1, device=DEV) / C ** 0.5, torch.randn(sq, device=DEV)
    w2, b2 = torch.randn(C, sq, 1, 1, device=DEV) / sq ** 0.5, torch.randn(C, device=DEV)
    res = []
    for use in (False, True):
        bn = torch.nn.BatchNorm2d(C, momentum=0.01, eps=1e-3).to(DEV)
        x = x0.clone().requires_grad_(True)
        y = nn_ops.depthwise_conv2d(x, wd, 1, (1, 1, 1, 1), bn_stats=use)
        assert (conv.bn_partials(y) is not None) == use
        out = nn_ops.bn_swish_squeeze_excite(y, bn, w1, b1, w2, b2)
        out.backward(torch.randn(out.shape, generator=torch.Generator().manual_seed(2)).to(DEV))
        res.append((out.detach(), bn.running_mean.clone(), bn.running_var.clone(), x.grad,
                    bn.weight.grad, bn.bias.grad))
    for a, b in zip(*res):
        assert rel_l2(b, a.double()) < 1e-6
