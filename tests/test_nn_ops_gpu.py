"""e2ep BN / resize / depthwise / pooling / SE kernels vs an fp64 CPU reference of the same
PyTorch op (values, gradients, running statistics)."""
import pytest
import torch
import torch.nn.functional as F
from torch import nn

from helpers import rel_l2

pytestmark = pytest.mark.gpu
DEV = "cuda"


def _g(seed):
    return torch.Generator().manual_seed(seed)


@pytest.mark.parametrize("act", [None, "relu", "swish"])
@pytest.mark.parametrize("res", [False, True])
def test_bn_act_narrow_blocks(act, res):
    """e2ep_tune key 25 = 1: the single-launch BN of channels with 4097..8192 elements
    (32 x 16 x 16 here) on 256-thread blocks of 8 float4 per thread (the default, key 25 = 2,
    runs 512 x 4 and is covered by test_bn_act's (32, 24, 16, 16) case), train and eval, vs
    fp64."""
    from e2ep_amd import _lib
    lib = _lib.load()
    prev = lib.e2ep_tune(25, 1)
    try:
        for train in (True, False):
            test_bn_act(train, act, res, (32, 24, 16, 16), 1)
    finally:
        lib.e2ep_tune(25, prev)


@pytest.fixture(params=[0, 3], ids=["dw_grid_default", "dw_grid_3"])
def dw_grid(request):
    """Depthwise forward grid cap (e2ep_tune key 24): default, and 3 blocks so each wave walks
    many units of the grid-stride loop (with the fused BN input transform changing channel
    from unit to unit)."""
    from e2ep_amd import _lib
    if not request.param:
        yield 0
        return
    prev = _lib.load().e2ep_tune(24, request.param)
    yield request.param
    _lib.load().e2ep_tune(24, prev)


@pytest.fixture(params=[1, 0], ids=["bn_one_launch", "bn_split"])
def bn_path(request):
    """Run a BN test through the single-launch block-per-channel kernels (channels of
    N*H*W <= 32768) and again with every shape forced onto the split stats + apply kernels."""
    from e2ep_amd import _lib
    prev = _lib.call_raw("e2ep_bn_small", request.param)
    yield request.param
    _lib.call_raw("e2ep_bn_small", prev)


@pytest.mark.parametrize("train", [True, False])
@pytest.mark.parametrize("act", [None, "relu", "swish"])
@pytest.mark.parametrize("res", [False, True])
@pytest.mark.parametrize("shape", [(4, 24, 32, 32), (3, 7, 5, 9), (32, 6, 1, 1),
                                   (4, 160, 8, 8), (16, 128, 32, 32), (8, 16, 64, 64),
                                   (3, 12, 44, 36), (2, 8, 136, 128), (32, 24, 16, 16)])
def test_bn_act(train, act, res, shape, bn_path):
    from e2ep_amd import nn_ops
    g = _g(sum(shape) + 3 * train)
    x = torch.randn(*shape, generator=g) * 2 + 0.5
    r = torch.randn(*shape, generator=g) if res else None
    dy = torch.randn(*shape, generator=g)
    C = shape[1]
    bn = nn.BatchNorm2d(C, momentum=0.01, eps=1e-3)
    with torch.no_grad():
        bn.weight.copy_(1 + 0.3 * torch.randn(C, generator=g))
        bn.bias.copy_(0.2 * torch.randn(C, generator=g))
        bn.running_mean.copy_(0.1 * torch.randn(C, generator=g))
        bn.running_var.copy_(0.5 + torch.rand(C, generator=g))
    bn64 = nn.BatchNorm2d(C, momentum=0.01, eps=1e-3).double()
    bn64.load_state_dict(bn.state_dict())
    bn.train(train), bn64.train(train)
    bnd = bn.to(DEV)
    xd = x.to(DEV).requires_grad_(True)
    rd = r.to(DEV).requires_grad_(True) if res else None
    y = nn_ops.batch_norm_act(xd, bnd, act, rd)
    y.backward(dy.to(DEV))
    x64 = x.double().requires_grad_(True)
    r64 = r.double().requires_grad_(True) if res else None
    z = bn64(x64) + (r64 if res else 0)
    y64 = {None: z, "relu": torch.relu(z) if act == "relu" else z, "swish": z * torch.sigmoid(z)}[act]
    if act == "relu":
        y64 = torch.relu(z)
    y64.backward(dy.double())
    assert rel_l2(y, y64) < 1e-6
    assert rel_l2(xd.grad, x64.grad) < 1e-5
    assert rel_l2(bnd.weight.grad, bn64.weight.grad) < 1e-5
    assert rel_l2(bnd.bias.grad, bn64.bias.grad) < 1e-5
    if res:
        assert rel_l2(rd.grad, r64.grad) < 1e-6
    assert rel_l2(bnd.running_mean, bn64.running_mean) < 1e-6
    assert rel_l2(bnd.running_var, bn64.running_var) < 1e-6
    assert int(bnd.num_batches_tracked) == int(bn64.num_batches_tracked)


@pytest.mark.parametrize("shape", [(8, 24, 16, 16), (6, 10, 5, 7), (16, 136, 8, 8)])
def test_bn_drop_connect_fused(shape, bn_path):
    """MBConv tail in training: bn2 -> efficientnet-pytorch drop_connect (x / keep *
    floor(keep + u)) -> + inputs, fused into the BN kernels; vs fp64 torch."""
    from e2ep_amd import nn_ops
    g = _g(sum(shape))
    N, C = shape[:2]
    x = torch.randn(*shape, generator=g) * 2 + 0.5
    r = torch.randn(*shape, generator=g)
    dy = torch.randn(*shape, generator=g)
    u = torch.rand(N, generator=g)
    keep = 0.8
    bn = nn.BatchNorm2d(C, momentum=0.01, eps=1e-3)
    with torch.no_grad():
        bn.weight.copy_(1 + 0.3 * torch.randn(C, generator=g))
        bn.bias.copy_(0.2 * torch.randn(C, generator=g))
    bn64 = nn.BatchNorm2d(C, momentum=0.01, eps=1e-3).double()
    bn64.load_state_dict(bn.state_dict())
    bnd = bn.to(DEV).train()
    xd = x.to(DEV).requires_grad_(True)
    rd = r.to(DEV).requires_grad_(True)
    y = nn_ops.batch_norm_act(xd, bnd, None, rd, dc_rand=u.to(DEV), dc_keep=keep)
    y.backward(dy.to(DEV))
    x64 = x.double().requires_grad_(True)
    r64 = r.double().requires_grad_(True)
    mask = torch.floor(torch.tensor(keep, dtype=torch.float32) + u).double().view(N, 1, 1, 1)
    assert 0 < mask.sum() < N or N < 8  # the draw exercises both kept and dropped samples
    y64 = bn64(x64) / keep * mask + r64
    y64.backward(dy.double())
    assert rel_l2(y, y64) < 1e-6
    assert rel_l2(xd.grad, x64.grad) < 1e-5
    assert rel_l2(rd.grad, r64.grad) < 1e-6
    assert rel_l2(bnd.weight.grad, bn64.weight.grad) < 1e-5
    assert rel_l2(bnd.bias.grad, bn64.bias.grad) < 1e-5


@pytest.mark.parametrize("case", [((8, 65, 200, 200), (256, 256), None), ((4, 64, 16, 16), None, 2),
                                  ((2, 64, 128, 128), (200, 200), None), ((32, 64, 1, 1), (16, 16), None),
                                  ((3, 5, 17, 9), (40, 7), None), ((2, 7, 50, 60), (40, 90), None)])
def test_resize(case):
    from e2ep_amd import nn_ops
    shape, size, sf = case
    g = _g(shape[2] + shape[3])
    x = torch.randn(*shape, generator=g)
    xd = x.to(DEV).requires_grad_(True)
    y = nn_ops.resize(xd, size=size, scale_factor=sf)
    dy = torch.randn(y.shape, generator=g)
    y.backward(dy.to(DEV))
    x64 = x.double().requires_grad_(True)
    y64 = F.interpolate(x64, size=size, scale_factor=sf, mode="bilinear", align_corners=False)
    y64.backward(dy.double())
    assert y.shape == y64.shape
    # coordinates are computed in fp32 as PyTorch's own fp32 kernel does: compare to that
    # tightly, and to fp64 (different interpolation weights in the last bits) loosely
    y32 = F.interpolate(x, size=size, scale_factor=sf, mode="bilinear", align_corners=False)
    assert rel_l2(y, y32) < 1e-6
    assert rel_l2(y, y64) < 2e-5
    assert rel_l2(xd.grad, x64.grad) < 2e-5


@pytest.mark.parametrize("shape,out", [((2, 8, 50, 60), (40, 92)), ((2, 65, 200, 200), (256, 256)),
                                       ((1, 3, 128, 128), (200, 200))])
def test_resize_fwd_vector_path_bitwise(shape, out):
    """e2ep_resize_fwd's four-outputs-per-thread kernel (k_resize_fwd4: Wo % 4 == 0 and a 16-B
    aligned y) equals the one-output kernel (taken for a y one float off alignment) bitwise."""
    from e2ep_amd import _lib
    N, C, Hi, Wi = shape
    Ho, Wo = out
    x = torch.randn(*shape, generator=_g(Hi + Wo)).to(DEV)
    n = N * C * Ho * Wo
    buf = torch.full((n + 4,), float("nan"), device=DEV)
    ys = []
    for off in (0, 1):  # aligned: k_resize_fwd4; one float off: k_resize_fwd
        y = buf[off:off + n]
        _lib.call("e2ep_resize_fwd", _lib.ptr(x), N, C, C * Hi * Wi, Hi, Wi, Ho, Wo, Hi / Ho, Wi / Wo,
                  _lib.ptr(y), C * Ho * Wo, _lib.stream())
        ys.append(y.clone())
    assert torch.equal(ys[0], ys[1])
    y32 = F.interpolate(x.cpu(), size=out, mode="bilinear", align_corners=False)
    assert rel_l2(ys[0].view(N, C, Ho, Wo), y32) < 1e-6


@pytest.mark.parametrize("case", [(4, 144, 64, 64, 3, 2, (0, 1, 0, 1)), (4, 48, 32, 32, 3, 1, (1, 1, 1, 1)),
                                  (4, 192, 32, 32, 5, 2, (2, 2, 2, 2)), (2, 672, 16, 16, 5, 1, (2, 2, 2, 2)),
                                  (3, 8, 13, 11, 3, 2, (0, 1, 0, 1)), (2, 24, 128, 128, 3, 1, (1, 1, 1, 1)),
                                  (2, 8, 128, 128, 3, 2, (0, 1, 0, 1)), (2, 32, 64, 64, 3, 1, (1, 1, 1, 1)),
                                  (2, 40, 32, 32, 5, 1, (2, 2, 2, 2)), (3, 16, 16, 16, 3, 1, (1, 1, 1, 1)),
                                  (2, 12, 24, 20, 5, 1, (2, 2, 2, 2)), (2, 16, 32, 32, 5, 2, (1, 2, 1, 2)),
                                  (2, 8, 20, 24, 3, 2, (0, 1, 0, 1)), (2, 6, 64, 48, 5, 2, (2, 2, 2, 2)),
                                  (2, 16, 32, 32, 5, 1, (3, 1, 3, 1))])
@pytest.mark.parametrize("variant", [(2, 0), (1, 3)])
def test_depthwise(case, variant):
    """variant = (e2ep_tune key 23, key 24): the strip kernels' LDS window reads (2 = 16-B
    vector reads from the aligned boundary OFF = -pad_left mod 4 floats back, 1 = scalar
    reads) and the forward grid cap (0 = default; 3 blocks = every wave walks many units of
    the software-pipelined grid-stride loop)."""
    from e2ep_amd import _lib, ops
    lib = _lib.load()
    rows, blocks = variant
    prev = lib.e2ep_tune(23, rows)
    prevb = lib.e2ep_tune(24, blocks) if blocks else None
    try:
        _depthwise_case(ops, case)
    finally:
        lib.e2ep_tune(23, prev)
        if blocks:
            lib.e2ep_tune(24, prevb)


@pytest.mark.parametrize("case", [(4, 48, 32, 32, 3, 1, (1, 1, 1, 1)), (2, 672, 16, 16, 5, 1, (2, 2, 2, 2)),
                                  (2, 24, 128, 128, 3, 1, (1, 1, 1, 1)), (2, 32, 64, 64, 3, 1, (1, 1, 1, 1)),
                                  (2, 40, 32, 32, 5, 1, (2, 2, 2, 2)), (3, 16, 16, 16, 3, 1, (1, 1, 1, 1)),
                                  (2, 12, 24, 20, 5, 1, (2, 2, 2, 2)), (32, 192, 32, 32, 5, 1, (2, 2, 2, 2)),
                                  (32, 96, 64, 64, 3, 1, (1, 1, 1, 1)),
                                  # stride 2 (k_dw_bwd_pair_s2): K 3 pad-left 0 / 1, K 5 pad-left 1 / 2
                                  (4, 144, 64, 64, 3, 2, (0, 1, 0, 1)), (2, 16, 32, 32, 3, 2, (1, 1, 1, 1)),
                                  (4, 192, 32, 32, 5, 2, (2, 2, 2, 2)), (2, 16, 32, 32, 5, 2, (1, 2, 1, 2)),
                                  (8, 144, 128, 128, 3, 2, (0, 1, 0, 1)), (2, 6, 64, 48, 5, 2, (2, 2, 2, 2))])
@pytest.mark.parametrize("fused", [False, True], ids=["dw", "bn_swish_dw"])
def test_depthwise_bwd_pair_bitwise_equals_two_launches(case, fused):
    """e2ep_dwconv_bwd (data and weight gradient in one k_dw_bwd_pair / k_dw_bwd_pair_s2 launch) == the forked
    e2ep_dwconv_dgrad + e2ep_dwconv_wgrad, bitwise, for the plain depthwise conv and the
    MBConv _bn0 -> swish -> depthwise form (the weight gradient's input transform)."""
    from e2ep_amd import _lib, nn_ops, ops
    N, C, H, W, K, s, pad = case
    lib = _lib.load()
    P, Q = (H + pad[2] + pad[3] - K) // s + 1, (W + pad[0] + pad[1] - K) // s + 1
    assert lib.e2ep_dwconv_bwd_pair_ok(_lib.dims((N, C, H, W, K, P, Q, s, pad[2], pad[0]))) == 1
    # the large stride-2 layer stays on two forked launches (DW_S2_PAIR_UNITS)
    big = (32, 144, 128, 128, 3, 64, 64, 2, 0, 0)
    assert lib.e2ep_dwconv_bwd_pair_ok(_lib.dims(big)) == 0
    g = _g(C + H + 5)
    x = (torch.randn(N, C, H, W, generator=g) * 2 + 0.5).to(DEV)
    w = (torch.randn(C, 1, K, K, generator=g) / K).to(DEV)
    dy = torch.randn(N, C, P, Q, generator=g).to(DEV)
    bn = nn.BatchNorm2d(C, momentum=0.01, eps=1e-3).to(DEV)

    def run():
        xd, wd = x.clone().requires_grad_(True), w.clone().requires_grad_(True)
        bn.zero_grad()
        if fused:
            y = nn_ops.bn_act_depthwise_conv2d(xd, bn, "swish", wd, s, pad)
        else:
            y = ops.conv2d(xd, wd, None, s, pad, 1, groups=C)
        y.backward(dy)
        out = [xd.grad.clone(), wd.grad.clone()]
        if fused:
            out += [bn.weight.grad.clone(), bn.bias.grad.clone()]
        return out

    prev = nn_ops.set_dw_pair(False)
    try:
        two = run()
        nn_ops.set_dw_pair(True)
        one = run()
    finally:
        nn_ops.set_dw_pair(prev)
    assert all(torch.equal(a, c) for a, c in zip(one, two))


def _depthwise_case(ops, case):
    N, C, H, W, K, s, pad = case
    g = _g(C + H)
    x = torch.randn(N, C, H, W, generator=g)
    w = torch.randn(C, 1, K, K, generator=g) / K
    xd = x.to(DEV).requires_grad_(True)
    wd = w.to(DEV).requires_grad_(True)
    y = ops.conv2d(xd, wd, None, s, pad, 1, groups=C)
    dy = torch.randn(y.shape, generator=g)
    y.backward(dy.to(DEV))
    x64 = x.double().requires_grad_(True)
    w64 = w.double().requires_grad_(True)
    y64 = F.conv2d(F.pad(x64, pad), w64, None, s, 0, 1, C)
    y64.backward(dy.double())
    assert y.shape == y64.shape
    assert rel_l2(y, y64) < 1e-6
    assert rel_l2(xd.grad, x64.grad) < 1e-6
    assert rel_l2(wd.grad, w64.grad) < 1e-5


@pytest.mark.parametrize("case", [(4, 144, 64, 64, 3, 2, (0, 1, 0, 1), True),
                                  (2, 192, 32, 32, 5, 1, (2, 2, 2, 2), True),
                                  (2, 40, 32, 32, 5, 2, (1, 2, 1, 2), False),
                                  (3, 8, 13, 11, 3, 2, (0, 1, 0, 1), True),
                                  (2, 6, 64, 48, 5, 2, (2, 2, 2, 2), True),
                                  (8, 144, 128, 128, 3, 2, (0, 1, 0, 1), True),
                                  (8, 192, 64, 64, 3, 1, (1, 1, 1, 1), True),
                                  (8, 336, 32, 32, 5, 1, (2, 2, 2, 2), True)])
def test_bn_swish_depthwise_fused(case, bn_path, dw_grid):
    """MBConv _bn0 -> swish -> _depthwise_conv with the BN + swish applied inside the
    depthwise input load (e2ep_bn_stats + dwconv in_scale/in_shift), train and eval, vs fp64
    torch: output, x / gamma / beta / weight gradients and running statistics."""
    from e2ep_amd import nn_ops
    N, C, H, W, K, s, pad, train = case
    g = _g(C + H + K)
    x = torch.randn(N, C, H, W, generator=g) * 2 + 0.5
    w = torch.randn(C, 1, K, K, generator=g) / K
    bn = nn.BatchNorm2d(C, momentum=0.01, eps=1e-3)
    with torch.no_grad():
        bn.weight.copy_(1 + 0.3 * torch.randn(C, generator=g))
        bn.bias.copy_(0.2 * torch.randn(C, generator=g))
        bn.running_mean.copy_(0.1 * torch.randn(C, generator=g))
        bn.running_var.copy_(0.5 + torch.rand(C, generator=g))
    bn64 = nn.BatchNorm2d(C, momentum=0.01, eps=1e-3).double()
    bn64.load_state_dict(bn.state_dict())
    bn.train(train), bn64.train(train)
    bnd = bn.to(DEV)
    xd = x.to(DEV).requires_grad_(True)
    wd = w.to(DEV).requires_grad_(True)
    y = nn_ops.bn_act_depthwise_conv2d(xd, bnd, "swish", wd, s, pad)
    dy = torch.randn(y.shape, generator=g)
    y.backward(dy.to(DEV))
    x64 = x.double().requires_grad_(True)
    w64 = w.double().requires_grad_(True)
    z = bn64(x64)
    y64 = F.conv2d(F.pad(z * torch.sigmoid(z), pad), w64, None, s, 0, 1, C)
    y64.backward(dy.double())
    assert y.shape == y64.shape
    assert rel_l2(y, y64) < 1e-6
    assert rel_l2(xd.grad, x64.grad) < 1e-5
    assert rel_l2(wd.grad, w64.grad) < 1e-5
    assert rel_l2(bnd.weight.grad, bn64.weight.grad) < 1e-5
    assert rel_l2(bnd.bias.grad, bn64.bias.grad) < 1e-5
    assert rel_l2(bnd.running_mean, bn64.running_mean) < 1e-6
    assert rel_l2(bnd.running_var, bn64.running_var) < 1e-6
    assert int(bnd.num_batches_tracked) == int(bn64.num_batches_tracked)


def test_maxpool_avgpool_segate():
    from e2ep_amd import nn_ops
    g = _g(5)
    x = torch.randn(2, 16, 33, 64, generator=g)
    x[0, 0, :4, :4] = 1.0  # ties: first maximum wins
    xd = x.to(DEV).requires_grad_(True)
    y = nn_ops.max_pool3s2(xd)
    dy = torch.randn(y.shape, generator=g)
    y.backward(dy.to(DEV))
    x64 = x.double().requires_grad_(True)
    y64 = F.max_pool2d(x64, 3, 2, 1)
    y64.backward(dy.double())
    assert torch.equal(y.cpu().double(), y64) and rel_l2(xd.grad, x64.grad) < 1e-7
    # global average pool + SE gate
    a = torch.randn(2, 16, 1, 1, generator=g)
    xd = x.to(DEV).requires_grad_(True)
    ad = a.to(DEV).requires_grad_(True)
    out = nn_ops.se_gate(xd, ad) + nn_ops.global_avg_pool(xd)
    dy = torch.randn(out.shape, generator=g)
    out.backward(dy.to(DEV))
    x64 = x.double().requires_grad_(True)
    a64 = a.double().requires_grad_(True)
    o64 = x64 * torch.sigmoid(a64) + x64.mean((2, 3), keepdim=True)
    o64.backward(dy.double())
    assert rel_l2(out, o64) < 1e-6 and rel_l2(xd.grad, x64.grad) < 1e-6 and rel_l2(ad.grad, a64.grad) < 1e-6


def test_bev_stem_resize_conv_fused():
    """bev_stem(bev, tgt, w) == conv7x7/2(resize(cat(bev, tgt))) with grads for bev and w."""
    from e2ep_amd import bev_stem
    g = _g(77)
    bev = torch.randn(2, 64, 50, 50, generator=g)
    tgt = (torch.rand(2, 1, 50, 50, generator=g) > 0.9).float()
    w = torch.randn(64, 65, 7, 7, generator=g) / (65 * 49) ** 0.5
    bd = bev.to(DEV).requires_grad_(True)
    wd = w.to(DEV).requires_grad_(True)
    y = bev_stem.bev_stem(bd, tgt.to(DEV), wd, (64, 64))
    gy = torch.randn(y.shape, generator=g)
    y.backward(gy.to(DEV))
    b64 = bev.double().requires_grad_(True)
    w64 = w.double().requires_grad_(True)
    x = F.interpolate(torch.cat([b64, tgt.double()], 1), size=(64, 64), mode="bilinear", align_corners=False)
    y64 = F.conv2d(x, w64, None, 2, 3)
    y64.backward(gy.double())
    assert rel_l2(y, y64) < 2e-5
    assert rel_l2(bd.grad, b64.grad) < 2e-5
    assert rel_l2(wd.grad, w64.grad) < 2e-5


@pytest.mark.parametrize("N,C,Hi,Wi,Ho,Wo", [(2, 64, 200, 200, 256, 256), (3, 70, 37, 45, 50, 61),
                                             (1, 5, 9, 33, 9, 40)])
def test_resize_bwd_channels_last_equals_nchw(N, C, Hi, Wi, Ho, Wo):
    """e2ep_resize_bwd_cl (pillar-major output for the lift-splat backward) is bit-equal to the
    NCHW gather backward, transposed to channels-last."""
    from e2ep_amd import _lib
    g = torch.randn(N, C, Ho, Wo, generator=_g(C + Wi)).to(DEV)
    sh, sw = Hi / Ho, Wi / Wo
    ref = torch.empty(N, C, Hi, Wi, device=DEV)
    ws = torch.empty(N * C * Ho * Wi, device=DEV)
    _lib.call("e2ep_resize_bwd", _lib.ptr(g), Ho * Wo, N * C, Hi, Wi, Ho, Wo, sh, sw,
              _lib.ptr(ref), 0, _lib.ptr(ws), _lib.stream())
    out = torch.empty(N, C, Hi, Wi, device=DEV, memory_format=torch.channels_last)
    _lib.call("e2ep_resize_bwd_cl", _lib.ptr(g), Ho * Wo, N, C, Hi, Wi, Ho, Wo, sh, sw,
              _lib.ptr(out), _lib.stream())
    assert torch.equal(out, ref)


def test_lift_splat_bwd_takes_channels_last_gradient():
    """The lift-splat backward fed a channels-last BEV gradient (no transpose) returns exactly
    the gradients it returns for the same gradient in NCHW."""
    from e2ep_amd import lss, synthetic
    from model.bev_model import BevModel
    from tool.config import default_cfg
    bm = BevModel(default_cfg()).to(DEV)
    K, E = synthetic.rig(4, 256)
    plan = bm.plan(K.unsqueeze(0).expand(2, *K.shape).contiguous(),
                   E.unsqueeze(0).expand(2, *E.shape).contiguous(), DEV)
    gen = _g(5)
    prob = torch.rand(8, plan.D, plan.h, plan.w, generator=gen).softmax(1).to(DEV)
    feat = torch.randn(8, 64, plan.h, plan.w, generator=gen).to(DEV)
    gbev = torch.randn(2, 64, plan.X, plan.Y, generator=gen).to(DEV)
    grads = []
    for gb in (gbev.contiguous(), gbev.contiguous(memory_format=torch.channels_last)):
        p, f = prob.clone().requires_grad_(True), feat.clone().requires_grad_(True)
        lss.lift_splat(p, f, plan).backward(gb)
        grads.append((p.grad, f.grad))
    assert torch.equal(grads[0][0], grads[1][0]) and torch.equal(grads[0][1], grads[1][1])


@pytest.mark.parametrize("shape", [(8, 96, 16, 16, 6), (4, 40, 9, 7, 10), (32, 672, 16, 16, 28),
                                   (32, 1632, 8, 8, 68), (5, 300, 3, 3, 75), (2, 4096, 2, 2, 256),
                                   (3, 68, 17, 4, 8), (7, 36, 5, 5, 9), (3, 42, 10, 10, 7),
                                   (32, 960, 16, 16, 40)])
def test_squeeze_excite_fused(shape):
    """Fused SE (pool -> 1x1 -> swish -> 1x1 -> sigmoid gate) vs fp64 torch, all gradients,
    incl. excite workgroups straddling up to 17 planes (HW = 68), scalar planes (HW = 25) and
    C % 4 != 0 (C = 42); bitwise deterministic run to run."""
    from e2ep_amd import nn_ops
    N, C, H, W, sq = shape
    g = _g(C + sq)
    x = torch.randn(N, C, H, W, generator=g)
    w1 = torch.randn(sq, C, 1, 1, generator=g) / C ** 0.5
    b1 = torch.randn(sq, generator=g) * 0.1
    w2 = torch.randn(C, sq, 1, 1, generator=g) / sq ** 0.5
    b2 = torch.randn(C, generator=g) * 0.1
    dy = torch.randn(N, C, H, W, generator=g)
    ts = [t.to(DEV).requires_grad_(True) for t in (x, w1, b1, w2, b2)]
    y = nn_ops.squeeze_excite(*ts)
    y.backward(dy.to(DEV))
    rs = [t.double().requires_grad_(True) for t in (x, w1, b1, w2, b2)]
    p = F.adaptive_avg_pool2d(rs[0], 1)
    h = F.conv2d(p, rs[1], rs[2])
    h = h * torch.sigmoid(h)
    a = F.conv2d(h, rs[3], rs[4])
    y64 = rs[0] * torch.sigmoid(a)
    y64.backward(dy.double())
    assert rel_l2(y, y64) < 1e-6
    for got, ref in zip(ts, rs):
        assert rel_l2(got.grad, ref.grad) < 1e-5
    ts2 = [t.detach().clone().requires_grad_(True) for t in ts]
    y2 = nn_ops.squeeze_excite(*ts2)
    y2.backward(dy.to(DEV))
    assert torch.equal(y, y2)
    for a, b in zip(ts, ts2):
        assert torch.equal(a.grad, b.grad)


@pytest.fixture(params=[True, False], ids=["bn_sums_in_se", "bn_own_reduce"])
def se_bn_sums(request):
    """The split-path _bn1 backward with its channel sums from the SE's da pass
    (e2ep_se_bwd_bn + e2ep_bn_bwd_planes), and with its own reduction (e2ep_bn_bwd)."""
    from e2ep_amd import nn_ops
    prev = nn_ops.set_se_bn_sums(request.param)
    yield request.param
    nn_ops.set_se_bn_sums(prev)


@pytest.mark.parametrize("case", [(8, 96, 16, 16, 6, True), (4, 40, 9, 7, 10, True),
                                  (32, 672, 16, 16, 28, True), (5, 300, 3, 3, 75, False),
                                  (2, 144, 64, 64, 6, True), (32, 144, 64, 64, 6, True),
                                  (32, 48, 128, 128, 12, True), (6, 56, 30, 30, 14, True)])
def test_bn_swish_se_fused(case, bn_path, se_bn_sums):
    """MBConv _bn1 -> swish -> SE with the BN + swish applied on load by the SE kernels
    (e2ep_bn_stats + se x_scale/x_shift; backward through e2ep_bn_bwd gate_logit /
    gate_dpooled, or on the split path e2ep_bn_bwd_planes with the sums from the SE pass),
    train and eval, vs fp64 torch: output, every gradient, running stats."""
    from e2ep_amd import nn_ops
    N, C, H, W, sq, train = case
    g = _g(C + sq + H)
    x = torch.randn(N, C, H, W, generator=g) * 2 + 0.5
    w1 = torch.randn(sq, C, 1, 1, generator=g) / C ** 0.5
    b1 = torch.randn(sq, generator=g) * 0.1
    w2 = torch.randn(C, sq, 1, 1, generator=g) / sq ** 0.5
    b2 = torch.randn(C, generator=g) * 0.1
    dy = torch.randn(N, C, H, W, generator=g)
    bn = nn.BatchNorm2d(C, momentum=0.01, eps=1e-3)
    with torch.no_grad():
        bn.weight.copy_(1 + 0.3 * torch.randn(C, generator=g))
        bn.bias.copy_(0.2 * torch.randn(C, generator=g))
        bn.running_mean.copy_(0.1 * torch.randn(C, generator=g))
        bn.running_var.copy_(0.5 + torch.rand(C, generator=g))
    bn64 = nn.BatchNorm2d(C, momentum=0.01, eps=1e-3).double()
    bn64.load_state_dict(bn.state_dict())
    bn.train(train), bn64.train(train)
    bnd = bn.to(DEV)
    ts = [t.to(DEV).requires_grad_(True) for t in (x, w1, b1, w2, b2)]
    y = nn_ops.bn_swish_squeeze_excite(ts[0], bnd, *ts[1:])
    y.backward(dy.to(DEV))
    rs = [t.double().requires_grad_(True) for t in (x, w1, b1, w2, b2)]
    z = bn64(rs[0])
    u = z * torch.sigmoid(z)
    h = F.conv2d(F.adaptive_avg_pool2d(u, 1), rs[1], rs[2])
    a = F.conv2d(h * torch.sigmoid(h), rs[3], rs[4])
    y64 = u * torch.sigmoid(a)
    y64.backward(dy.double())
    assert rel_l2(y, y64) < 1e-6
    for got, ref in zip(ts, rs):
        assert rel_l2(got.grad, ref.grad) < 1e-5
    assert rel_l2(bnd.weight.grad, bn64.weight.grad) < 1e-5
    assert rel_l2(bnd.bias.grad, bn64.bias.grad) < 1e-5
    assert rel_l2(bnd.running_mean, bn64.running_mean) < 1e-6
    assert rel_l2(bnd.running_var, bn64.running_var) < 1e-6


@pytest.mark.parametrize("rows,E,p", [(2048, 258, 0.1), (112, 258, 0.0), (37, 100, 0.5)])
def test_add_dropout_layernorm_fused(rows, E, p):
    """y = LayerNorm(a + dropout(b)) (transformer post-norm residual) vs fp64 torch, with the
    dropout mask given by explicit uniforms; gradients of a, b, gamma, beta."""
    from e2ep_amd import nn_ops
    g = _g(rows + E)
    a = torch.randn(rows, E, generator=g)
    b = torch.randn(rows, E, generator=g)
    u = torch.rand(rows, E, generator=g)
    gamma = 1 + 0.2 * torch.randn(E, generator=g)
    beta = 0.1 * torch.randn(E, generator=g)
    dy = torch.randn(rows, E, generator=g)
    ts = [t.to(DEV).requires_grad_(True) for t in (a, b, gamma, beta)]
    y = nn_ops._AddDropLN.apply(ts[0], ts[1], ts[2], ts[3], u.to(DEV) if p > 0 else None, None, p,
                                1e-5)
    y.backward(dy.to(DEV))
    rs = [t.double().requires_grad_(True) for t in (a, b, gamma, beta)]
    mask = (u >= p).double() / (1 - p) if p > 0 else torch.ones_like(u).double()
    y64 = F.layer_norm(rs[0] + rs[1] * mask, (E,), rs[2], rs[3], 1e-5)
    y64.backward(dy.double())
    assert rel_l2(y, y64) < 1e-6
    for got, ref in zip(ts, rs):
        assert rel_l2(got.grad, ref.grad) < 1e-5


@pytest.mark.parametrize("rows,E,p", [(2048, 258, 0.1), (112, 258, 0.1), (7, 33, 0.5)])
def test_add_dropout_layernorm_seeded(rows, E, p):
    """The seeded LayerNorm dropout (no uniform tensor) keeps element row*E + c exactly when the
    shared counter hash does: the mask comes from e2ep_attn_keep_mask over one (rows x E)
    'head', and values / all gradients match fp64 torch with that mask."""
    from e2ep_amd import _lib, nn_ops
    g = _g(rows * 3 + E)
    a = torch.randn(rows, E, generator=g)
    b = torch.randn(rows, E, generator=g)
    gamma = 1 + 0.2 * torch.randn(E, generator=g)
    beta = 0.1 * torch.randn(E, generator=g)
    dy = torch.randn(rows, E, generator=g)
    seed = torch.tensor([12345 + rows], dtype=torch.int32, device=DEV)
    keep = torch.empty(rows, E, dtype=torch.uint8, device=DEV)
    _lib.call("e2ep_attn_keep_mask", _lib.ptr(seed), 1, rows, E, p, _lib.ptr(keep), _lib.stream())
    keep = keep.cpu().double()
    assert abs(float(keep.mean()) - (1 - p)) < 0.05
    ts = [t.to(DEV).requires_grad_(True) for t in (a, b, gamma, beta)]
    norm = torch.nn.LayerNorm(E).to(DEV)
    norm.weight, norm.bias = torch.nn.Parameter(ts[2]), torch.nn.Parameter(ts[3])
    y = nn_ops.add_drop_layer_norm(ts[0], ts[1], norm, p, seed=seed)
    y.backward(dy.to(DEV))
    rs = [t.double().requires_grad_(True) for t in (a, b, gamma, beta)]
    y64 = F.layer_norm(rs[0] + rs[1] * keep / (1 - p), (E,), rs[2], rs[3], 1e-5)
    y64.backward(dy.double())
    assert rel_l2(y, y64) < 1e-6
    for got, ref in zip((ts[0], ts[1], norm.weight, norm.bias), rs):
        assert rel_l2(got.grad, ref.grad) < 1e-5
    y2 = nn_ops.add_drop_layer_norm(ts[0].detach(), ts[1].detach(), norm, p, seed=seed)
    assert torch.equal(y2, y.detach())


def test_dropout_seed_pool_hands_out_distinct_seeds():
    from e2ep_amd import rng
    rng.begin_step(DEV)
    seeds = [rng.seed(DEV) for _ in range(40)]
    vals = torch.cat(seeds).cpu().tolist()
    assert len(set(vals)) == 40 and all(s.numel() == 1 and s.dtype == torch.int32 for s in seeds)
    rng.begin_step(DEV)
    assert torch.cat([rng.seed(DEV) for _ in range(40)]).cpu().tolist() != vals
    rng.end_step()
    assert rng._pool is None  # later calls draw fresh seeds again


@pytest.mark.parametrize("shape", [(32, 48, 32, 32), (3, 5, 7, 9), (2, 1, 4, 4)])
def test_softmax_channels_vs_fp64(shape):
    """Depth softmax over channels (model/bev_model.py:64) vs torch fp64, values and grad."""
    from e2ep_amd import nn_ops
    g = _g(sum(shape))
    x = torch.randn(*shape, generator=g) * 3
    dy = torch.randn(*shape, generator=g)
    xd = x.to(DEV).requires_grad_(True)
    y = nn_ops.softmax_channels(xd)
    (y * dy.to(DEV)).sum().backward()
    x64 = x.double().requires_grad_(True)
    y64 = x64.softmax(1)
    (y64 * dy.double()).sum().backward()
    assert rel_l2(y.detach().cpu(), y64) < 1e-6
    assert rel_l2(xd.grad.cpu(), x64.grad) < 1e-5


@pytest.mark.parametrize("shapes", [[(4, 64, 16, 16)] * 5, [(3, 56, 32, 32), (3, 160, 32, 32)],
                                    [(2, 1, 2, 2), (2, 3, 2, 2), (2, 2, 2, 2)],
                                    [(2, 5, 4, 4)] * 8])
def test_cat_channels_matches_torch(shapes):
    """e2ep_cat_channels / e2ep_split_channels (ASPP and UpsamplingConcat concatenation) vs
    torch.cat and its gradient: bit-exact (pure data movement)."""
    from e2ep_amd import nn_ops
    g = _g(len(shapes))
    xs = [torch.randn(*s, generator=g) for s in shapes]
    xd = [x.to(DEV).requires_grad_(True) for x in xs]
    y = nn_ops.cat_channels(xd)
    assert torch.equal(y.detach().cpu(), torch.cat(xs, 1))
    dy = torch.randn(y.shape, generator=g)
    y.backward(dy.to(DEV))
    c0 = 0
    for x, s in zip(xd, shapes):
        assert x.grad.is_contiguous()
        assert torch.equal(x.grad.cpu(), dy[:, c0:c0 + s[1]])
        c0 += s[1]


def test_sum3_eq_mask_counters():
    """e2ep_sum3 = (a + b) + c in fp32 with gradient 1 to each; e2ep_eq_mask_i64 = tok == v on
    a row-strided token slice; e2ep_add_i64_multi adds to every counter in its table."""
    from e2ep_amd import _lib, nn_ops
    a, b, c = (torch.tensor(v, device=DEV, requires_grad=True) for v in (1.1, 2.0e-7, -3.3))
    s = nn_ops.sum3(a, b, c)
    assert s.item() == ((torch.tensor(1.1) + torch.tensor(2.0e-7)) + torch.tensor(-3.3)).item()
    s.backward()
    assert a.grad.item() == b.grad.item() == c.grad.item() == 1.0
    tok = torch.randint(0, 5, (6, 15), generator=_g(3))
    td = tok.to(DEV)[:, 1:]
    assert torch.equal(nn_ops.eq_mask(td, 2).cpu(), tok[:, 1:] == 2)
    ctr = [torch.full((), k, dtype=torch.int64, device=DEV) for k in range(300)]
    table = torch.tensor([t.data_ptr() for t in ctr], dtype=torch.int64, device=DEV)
    _lib.call("e2ep_add_i64_multi", _lib.ptr(table), len(ctr), 1, _lib.stream())
    assert [int(t) for t in ctr] == [k + 1 for k in range(300)]


def test_step_rng_draws():
    """e2ep_rng_draw: uniform floats in [0, 1) and non-negative int32 seeds, distinct between
    consecutive launches and between graph replays (the kernel advances its own counter)."""
    from e2ep_amd import _lib, rng
    st = torch.tensor([12345, 0], dtype=torch.int64, device=DEV)
    f = torch.empty(4096, device=DEV)
    iv = torch.empty(64, dtype=torch.int32, device=DEV)

    def draw():
        _lib.call("e2ep_rng_draw", _lib.ptr(st), f.numel(), _lib.ptr(f), iv.numel(), _lib.ptr(iv),
                  _lib.stream())

    draw()
    a, ai = f.clone(), iv.clone()
    assert 0.0 <= float(a.min()) and float(a.max()) < 1.0 and abs(float(a.mean()) - 0.5) < 0.03
    assert int(ai.min()) >= 0 and len(set(ai.tolist())) == 64
    draw()
    assert not torch.equal(a, f) and int(st[1]) == 2
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    g = torch.cuda.CUDAGraph()
    with torch.cuda.stream(s):
        with torch.cuda.graph(g):
            draw()
    torch.cuda.current_stream().wait_stream(s)
    g.replay()
    b = f.clone()
    g.replay()
    assert not torch.equal(b, f) and int(st[1]) == 4
    # the module-level pools: views of one launch, retired by end_step
    rng.begin_step(DEV)
    u = rng.uniform((22, 32), DEV)
    v = rng.uniform((8, 2), DEV)
    assert u.shape == (22, 32) and v.shape == (8, 2) and u.data_ptr() != v.data_ptr()
    rng.end_step()
    assert rng.uniform((3,), DEV).shape == (3,)


def test_sigmoid_swish_error_bound():
    """common.h sigmoid_f / swish_f (v_exp_f32 of the fp32-rounded -z log2(e), v_rcp_f32),
    used by every swish, swish derivative and SE gate of the BN / depthwise / SE kernels,
    against fp64 on the same fp32 z over [-90, 90] (the error grows with |z|, it
    is not "a few ulp"): relative error <= 2^-24 (2 |z| + 8) wherever sigmoid(z) is a normal fp32
    number (z > -87.3); below that the reciprocal's denormal result is flushed to 0, an
    absolute error under 2^-126 (sigmoid) / 91 * 2^-126 (swish).  Probed through
    e2ep_se_gate_fwd (x = 1: sigmoid(a)) and e2ep_act_fwd (swish); the measured worst ratio to
    the bound is printed and recorded."""
    import numpy as np
    from e2ep_amd import _lib
    from test_model_b8_gpu import _record
    z = torch.cat([torch.linspace(-90, 90, 1 << 20), torch.tensor([0.0, -0.0, 1e-30, -1e-30,
                   -87.2, -87.4, -87.9, -88.0, -88.7, -89.0, 87.9, 88.7])]).float()
    zd = z.to(DEV)
    n = z.numel()
    sig = torch.empty_like(zd)
    _lib.call("e2ep_se_gate_fwd", _lib.ptr(torch.ones_like(zd)), _lib.ptr(zd), n, 1,
              _lib.ptr(sig), _lib.stream())
    sw = torch.empty_like(zd)
    _lib.call("e2ep_act_fwd", _lib.ptr(zd), n, 2, _lib.ptr(sw), _lib.stream())
    z64 = z.double().numpy()
    ref_s = 1.0 / (1.0 + np.exp(-z64))
    ref_w = z64 * ref_s
    got_s, got_w = sig.cpu().double().numpy(), sw.cpu().double().numpy()
    tiny = 2.0 ** -126
    nrm = ref_s >= tiny
    # rounding -log2(e) z contributes |z| 2^-24; v_exp_f32 / v_rcp_f32 and the fp32 log2(e)
    # the rest (measured worst 3.9e-6 relative at z = -44.4: 1.13 x 2^-24 (|z| + 5))
    bound = 2.0 ** -24 * (2.0 * np.abs(z64) + 8.0)
    rs = np.abs(got_s - ref_s)[nrm] / ref_s[nrm]
    nz = nrm & (z64 != 0)
    rw = np.abs(got_w - ref_w)[nz] / np.abs(ref_w[nz])
    worst_s = float(np.max(rs / bound[nrm]))
    worst_w = float(np.max(rw / bound[nz]))
    at = float(z64[nrm][np.argmax(rs / bound[nrm])])
    print(f"sigmoid_f worst rel err / bound {worst_s:.3f} (at z = {at:.3f}), swish_f "
          f"{worst_w:.3f}; max rel {rs.max():.3e} / {rw.max():.3e}")
    _record("activation", "sigmoid_swish_vs_fp64", sigmoid_worst_over_bound=worst_s,
            swish_worst_over_bound=worst_w, sigmoid_max_rel=float(rs.max()),
            swish_max_rel=float(rw.max()), worst_at_z=at)
    assert worst_s <= 1.0 and worst_w <= 1.0
    assert np.all(np.abs(got_s - ref_s)[~nrm] <= tiny)
    assert np.all(np.abs(got_w - ref_w)[~nrm] <= 91 * tiny)
    assert got_w[z64 == 0].tolist() == [0.0, 0.0]
