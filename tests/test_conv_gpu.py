"""e2ep implicit-GEMM conv (fp32 MFMA) vs an fp64 CPU reference of the same op, for every
conv geometry family of the ParkingModel hot path."""
import pytest
import torch
import torch.nn.functional as F

from helpers import rel_l2

pytestmark = pytest.mark.gpu
DEV = "cuda"

# (N, Cin, H, W, Cout, R, S, stride, pad(l,r,t,b), dil, bias, act)
CASES = [
    (2, 65, 64, 64, 64, 7, 7, 2, (3, 3, 3, 3), 1, False, 0),     # BEV conv1 (reduced H)
    (2, 64, 16, 16, 64, 3, 3, 1, (1, 1, 1, 1), 1, False, 1),     # BasicBlock 3x3 (+relu)
    (2, 64, 16, 16, 128, 3, 3, 2, (1, 1, 1, 1), 1, False, 0),    # layer2 stride-2
    (2, 64, 16, 16, 128, 1, 1, 2, (0, 0, 0, 0), 1, False, 0),    # downsample 1x1/2
    (4, 3, 32, 32, 48, 3, 3, 2, (0, 1, 0, 1), 1, False, 0),      # EfficientNet stem SAME pad
    (4, 160, 16, 16, 64, 3, 3, 1, (12, 12, 12, 12), 12, False, 0),  # ASPP dilation 12
    (4, 160, 16, 16, 64, 3, 3, 1, (24, 24, 24, 24), 24, False, 0),  # ASPP dilation 24
    (4, 320, 16, 16, 64, 1, 1, 1, (0, 0, 0, 0), 1, False, 0),    # ASPP project
    (4, 64, 16, 16, 160, 1, 1, 1, (0, 0, 0, 0), 1, True, 0),     # DeepLab last 1x1 + bias
    (4, 216, 32, 32, 48, 3, 3, 1, (1, 1, 1, 1), 1, False, 0),    # UpsamplingConcat
    (8, 144, 1, 1, 6, 1, 1, 1, (0, 0, 0, 0), 1, True, 0),        # SE reduce (1x1 map)
    (8, 6, 1, 1, 144, 1, 1, 1, (0, 0, 0, 0), 1, True, 0),        # SE expand
    (2, 64, 50, 50, 3, 1, 1, 1, (0, 0, 0, 0), 1, True, 0),       # seg-head classifier
    (3, 24, 33, 17, 40, 5, 5, 2, (2, 2, 2, 2), 1, False, 1),     # odd sizes, k5/s2
    (4, 24, 32, 32, 144, 1, 1, 1, (0, 0, 0, 0), 1, False, 0),    # MBConv expand (1x1 wgrad path)
    (3, 100, 8, 8, 70, 1, 1, 1, (0, 0, 0, 0), 1, False, 0),      # 1x1, partial 32-tiles
    (2, 336, 24, 24, 56, 1, 1, 1, (0, 0, 0, 0), 1, False, 0),    # MBConv project
    (2, 64, 20, 20, 3, 1, 1, 1, (0, 0, 0, 0), 1, True, 0),       # 1x1 to 3 channels + bias
    (2, 64, 24, 24, 64, 3, 3, 1, (1, 1, 1, 1), 1, False, 1),     # 3x3 s1 (tap wgrad path)
    (2, 40, 16, 16, 24, 3, 3, 1, (2, 2, 2, 2), 2, False, 0),     # dilated 3x3, partial tiles
    (2, 65, 20, 24, 48, 5, 5, 1, (2, 2, 2, 2), 1, True, 0),      # 5x5 s1
    (8, 32, 128, 128, 192, 1, 1, 1, (0, 0, 0, 0), 1, False, 0),  # 1x1 wgrad 64x32 wave tiles
    (16, 64, 128, 128, 24, 1, 1, 1, (0, 0, 0, 0), 1, False, 0),  # 1x1 wgrad 32x64 wave tiles
    (16, 64, 128, 128, 64, 1, 1, 1, (0, 0, 0, 0), 1, False, 0),  # 1x1 wgrad 64x64 wave tiles
    (4, 128, 32, 32, 120, 1, 1, 1, (0, 0, 0, 0), 1, False, 0),   # 1x1 on the LDS-tiled wgrad
    (2, 2, 17, 19, 40, 3, 3, 1, (1, 1, 1, 1), 1, True, 1),       # direct path: K=18, bias+relu
    (3, 24, 16, 16, 24, 1, 1, 1, (0, 0, 0, 0), 1, False, 0),     # direct fwd 1x1 K=24
    (2, 1, 30, 30, 64, 5, 5, 2, (2, 2, 2, 2), 1, False, 0),      # direct K=25, Cout=64, s2
    (2, 3, 21, 23, 17, 3, 3, 1, (2, 2, 2, 2), 2, False, 0),      # direct, dilated, ragged Cout
    (4, 160, 16, 16, 64, 3, 3, 1, (36, 36, 36, 36), 36, False, 0),  # ASPP dilation 36: 8 dead taps
    (2, 16, 9, 7, 24, 5, 5, 2, (9, 9, 9, 9), 3, False, 1),       # strided, dead taps both axes
    (2, 40, 6, 6, 32, 3, 3, 1, (6, 6, 6, 1), 6, True, 0),        # asymmetric pad: dead rows/cols
    (2, 65, 64, 64, 64, 7, 7, 2, (3, 3, 3, 3), 1, True, 1),      # stem: 49-row tail, bias+relu
    (2, 216, 20, 20, 64, 3, 3, 1, (1, 1, 1, 1), 1, False, 0),    # 8-channel remainder x 9 taps
    (1, 64, 40, 40, 48, 3, 3, 1, (1, 1, 1, 1), 1, False, 0),     # M = 48 (partial 64-row tile)
]


@pytest.fixture(params=[0, 1, 2, 3, 4], ids=["auto", "gemm1", "gemm2", "gemm2_128", "gemm1x1"])
def gemm_variant(request):
    """Conv GEMM selection (e2ep_conv_gemm_variant): automatic, the first-generation kernel
    everywhere, the second-generation forward / data-gradient kernel wherever it applies
    (256- or 128-column tiles), automatic with the 1x1 convs on the column-batched k_gemm."""
    from e2ep_amd import _lib
    old = _lib.call_raw("e2ep_conv_gemm_variant", request.param)
    yield request.param
    _lib.call_raw("e2ep_conv_gemm_variant", old)


@pytest.mark.parametrize("case", CASES, ids=[str(i) for i in range(len(CASES))])
def test_conv_fwd_bwd_vs_fp64(case, gemm_variant):
    from e2ep_amd import conv
    N, Cin, H, W, Cout, R, S, st, pad, dil, has_b, act = case
    g = torch.Generator().manual_seed(hash(case) & 0xFFFF)
    x = torch.randn(N, Cin, H, W, generator=g)
    w = torch.randn(Cout, Cin, R, S, generator=g) / (Cin * R * S) ** 0.5
    b = torch.randn(Cout, generator=g) if has_b else None
    xd = x.to(DEV).requires_grad_(True)
    wd = w.to(DEV).requires_grad_(True)
    bd = b.to(DEV).requires_grad_(True) if has_b else None
    y = conv.conv2d(xd, wd, bd, (st, st), pad, (dil, dil), act)
    gy = torch.randn(y.shape, generator=g)
    y.backward(gy.to(DEV))
    x64 = x.double().requires_grad_(True)
    w64 = w.double().requires_grad_(True)
    b64 = b.double().requires_grad_(True) if has_b else None
    y64 = F.conv2d(F.pad(x64, pad), w64, b64, st, 0, dil)
    if act:
        y64 = torch.relu(y64)
    y64.backward(gy.double())
    assert y.shape == y64.shape
    assert rel_l2(y, y64) < 2e-6
    assert rel_l2(xd.grad, x64.grad) < 2e-6
    assert rel_l2(wd.grad, w64.grad) < 2e-6
    if has_b:
        assert rel_l2(bd.grad, b64.grad) < 2e-6


@pytest.mark.parametrize("case", CASES, ids=[str(i) for i in range(len(CASES))])
def test_conv_wgrad_kstep32_vs_fp64(case):
    """The tiled weight-gradient kernel with 32-pixel K-steps (e2ep_conv_wgrad_kstep)."""
    from e2ep_amd import _lib, conv
    N, Cin, H, W, Cout, R, S, st, pad, dil, has_b, act = case
    g = torch.Generator().manual_seed(hash(case) & 0xFFFF)
    x = torch.randn(N, Cin, H, W, generator=g)
    w = torch.randn(Cout, Cin, R, S, generator=g) / (Cin * R * S) ** 0.5
    wd = w.to(DEV).requires_grad_(True)
    old = _lib.call_raw("e2ep_conv_wgrad_kstep", 32)
    try:
        y = conv.conv2d(x.to(DEV), wd, None, (st, st), pad, (dil, dil), 0)
        gy = torch.randn(y.shape, generator=g)
        y.backward(gy.to(DEV))
    finally:
        _lib.call_raw("e2ep_conv_wgrad_kstep", old)
    w64 = w.double().requires_grad_(True)
    F.conv2d(F.pad(x.double(), pad), w64, None, st, 0, dil).backward(gy.double())
    assert rel_l2(wd.grad, w64.grad) < 2e-6


def test_conv_wgrad_deterministic():
    from e2ep_amd import conv
    g = torch.Generator().manual_seed(0)
    x = torch.randn(8, 64, 32, 32, generator=g).to(DEV)
    w = (torch.randn(64, 64, 3, 3, generator=g) / 24).to(DEV)
    gy = torch.randn(8, 64, 32, 32, generator=g).to(DEV)
    outs = []
    for _ in range(2):
        wd = w.clone().requires_grad_(True)
        conv.conv2d(x, wd, None, (1, 1), (1, 1, 1, 1)).backward(gy)
        outs.append(wd.grad.clone())
    assert torch.equal(outs[0], outs[1])


# skip passthrough: the block input's skip-connection gradient is added inside the data
# gradient kernel (e2ep_conv_dgrad_acc), both without split-K (large maps) and with it
# (small maps -> k_conv_reduce adds it), plus the partial-channel (grad_channels) case.
SKIP_CASES = [
    (2, 24, 32, 32, 144, 1, 1, (0, 0, 0, 0), None),   # MBConv expand 1x1
    (2, 64, 16, 16, 64, 3, 3, (1, 1, 1, 1), None),    # BasicBlock conv1 3x3
    (2, 160, 8, 8, 960, 1, 1, (0, 0, 0, 0), None),    # small map: split-K data gradient
    (2, 65, 16, 16, 64, 3, 3, (1, 1, 1, 1), 64),      # grad_channels < Cin
]


@pytest.mark.parametrize("case", SKIP_CASES, ids=[str(i) for i in range(len(SKIP_CASES))])
def test_conv_skip_gradient_fused(case, gemm_variant):
    from e2ep_amd import conv
    N, Cin, H, W, Cout, R, S, pad, gc = case
    g = torch.Generator().manual_seed(17 + Cin)
    x = torch.randn(N, Cin, H, W, generator=g)
    w = torch.randn(Cout, Cin, R, S, generator=g) / (Cin * R * S) ** 0.5
    xd = x.to(DEV).requires_grad_(True)
    wd = w.to(DEV).requires_grad_(True)
    y, xs = conv.conv2d(xd, wd, None, (1, 1), pad, (1, 1), 0, grad_channels=gc, skip=True)
    gy = torch.randn(y.shape, generator=g)
    gs = torch.randn(x.shape, generator=g)
    ((y * gy.to(DEV)).sum() + (xs * gs.to(DEV)).sum()).backward()
    x64 = x.double().requires_grad_(True)
    w64 = w.double().requires_grad_(True)
    y64 = F.conv2d(F.pad(x64, pad), w64)
    (y64 * gy.double()).sum().backward()
    gx = x64.grad.clone()
    if gc is not None:
        gx[:, gc:] = 0
    gx += gs.double()
    assert rel_l2(y.detach().cpu(), y64) < 1e-5
    assert rel_l2(xd.grad.cpu(), gx) < 1e-5
    assert rel_l2(wd.grad.cpu(), w64.grad) < 1e-5


# low-precision operand modes (e2ep_amd.precision): against fp64 convolutions of the operands
# ROUNDED to bf16 / fp16 the kernels must agree to fp32-accumulation accuracy (the products
# are exact); against the unrounded fp64 result the error is the format's rounding (~3e-3
# bf16, ~4e-4 fp16 relative L2 at these depths) and is bounded loosely.
LP_CASES = [
    (2, 65, 64, 64, 64, 7, 7, 2, (3, 3, 3, 3), 1),      # BEV stem (tail rows)
    (2, 64, 40, 40, 64, 3, 3, 1, (1, 1, 1, 1), 1),      # 3x3 s1
    (4, 24, 32, 32, 144, 1, 1, 1, (0, 0, 0, 0), 1),     # MBConv expand (1x1)
    (4, 160, 16, 16, 64, 3, 3, 1, (12, 12, 12, 12), 12),  # ASPP dilated
    (2, 64, 16, 16, 128, 3, 3, 2, (1, 1, 1, 1), 1),     # stride 2 (dgrad phases)
    (8, 32, 128, 128, 48, 1, 1, 1, (0, 0, 0, 0), 1),    # 1x1, LDS-free weight gradient
]


@pytest.mark.parametrize("mode,dt,loose", [("bf16", torch.bfloat16, 1e-2), ("fp16", torch.float16, 2e-3)])
@pytest.mark.parametrize("case", LP_CASES, ids=[str(i) for i in range(len(LP_CASES))])
def test_conv_low_precision_operands(case, mode, dt, loose):
    from e2ep_amd import conv, precision
    N, Cin, H, W, Cout, R, S, st, pad, dil = case
    g = torch.Generator().manual_seed(31 + Cin)
    x = torch.randn(N, Cin, H, W, generator=g)
    w = torch.randn(Cout, Cin, R, S, generator=g) / (Cin * R * S) ** 0.5
    xd = x.to(DEV).requires_grad_(True)
    wd = w.to(DEV).requires_grad_(True)
    with precision.use(mode):
        assert precision.get() == mode
        y = conv.conv2d(xd, wd, None, (st, st), pad, (dil, dil), 0)
        gy = torch.randn(y.shape, generator=g)
        y.backward(gy.to(DEV))
    assert precision.get() == "fp32"
    r = lambda t: t.to(dt).double()  # noqa: E731
    y_r = F.conv2d(F.pad(r(x), pad), r(w), None, st, 0, dil)
    xr = r(x).requires_grad_(True)
    F.conv2d(F.pad(xr, pad), r(w), None, st, 0, dil).backward(r(gy))
    y64 = F.conv2d(F.pad(x.double(), pad), w.double(), None, st, 0, dil)
    assert rel_l2(y, y_r) < 2e-6                  # operands rounded, fp32 accumulation
    assert rel_l2(xd.grad, xr.grad) < 2e-6        # data gradient: gy and W rounded
    assert rel_l2(y, y64) < loose                 # vs the exact fp32-operand result
    if mode == "bf16":
        # C3 (bf16 forward / fp32 gradients, AMP-style): the weight-gradient GEMM takes bf16
        # operands too (x and gy rounded), accumulates and stores fp32
        wr = r(w).requires_grad_(True)
        F.conv2d(F.pad(r(x), pad), wr, None, st, 0, dil).backward(r(gy))
        assert rel_l2(wd.grad, wr.grad) < 5e-6
    else:
        # fp16 (inference mode C5): the weight gradient stays fp32 (exact-f32 MFMA)
        x64 = x.double().requires_grad_(True)
        w64 = w.double().requires_grad_(True)
        F.conv2d(F.pad(x64, pad), w64, None, st, 0, dil).backward(gy.double())
        assert rel_l2(wd.grad, w64.grad) < 2e-6


def test_tap_major_batch_one_launch_matches_per_weight():
    """TapMajorBatch: the first scope records the spatial weights (per-weight transposes), the
    second transposes all of them in one e2ep_transpose_multi launch; 1x1 weights pass
    through; a weight whose storage moved makes the next scope record again."""
    from e2ep_amd import conv
    torch.manual_seed(0)
    ws = [torch.randn(64, 65, 7, 7, device=DEV), torch.randn(48, 3, 3, 3, device=DEV),
          torch.randn(130, 70, 5, 5, device=DEV), torch.randn(32, 16, 1, 1, device=DEV)]
    ref = [w.permute(2, 3, 0, 1).reshape(w.shape[2] * w.shape[3], w.shape[0], w.shape[1]) for w in ws]
    tb = conv.TapMajorBatch()
    for it in range(3):
        with tb:
            outs = [conv.tap_major(w) for w in ws]
            assert (tb.recorded is not None) == (it > 0)
            torch.cuda.synchronize()
            for o, r in zip(outs[:3], ref[:3]):
                assert torch.equal(o, r)
            assert torch.equal(outs[3], ws[3])
    assert len(tb.recorded) == 3  # the 1x1 weight never enters the batch
    ws[2].data = ws[2].data.clone()  # same tensor object, storage moved (re-flattened)
    ref[2] = ref[2] * 1
    with tb:
        o = conv.tap_major(ws[2])
        torch.cuda.synchronize()
        assert torch.equal(o, ref[2])
    assert len(tb.recorded) == 1 and tb.recorded[0] is ws[2]


def test_side_stream_weight_gradient_equals_serial():
    """conv / linear / BEV-stem backward with the weight gradients forked to the side stream
    (conv._Fork) give bitwise the same gradients as the serial order (graph replay of the
    forked step: test_train_step_gpu / test_graph_gpu, graph == eager)."""
    from e2ep_amd import conv, nn_ops
    torch.manual_seed(3)
    x = torch.randn(8, 48, 32, 32, device=DEV, requires_grad=True)
    w = torch.randn(64, 48, 3, 3, device=DEV, requires_grad=True)
    b = torch.randn(64, device=DEV, requires_grad=True)
    lx = torch.randn(300, 258, device=DEV, requires_grad=True)
    lw = torch.randn(774, 258, device=DEV, requires_grad=True)
    lb = torch.randn(774, device=DEV, requires_grad=True)
    gy = torch.randn(8, 64, 32, 32, device=DEV)
    gl = torch.randn(300, 774, device=DEV)

    def run():
        for t in (x, w, b, lx, lw, lb):
            t.grad = None
        y = conv.conv2d(x, w, b, pad=(1, 1, 1, 1), act=1)
        yl = nn_ops.linear(lx, lw, lb)
        torch.autograd.backward([y, yl], [gy, gl])
        return [t.grad.clone() for t in (x, w, b, lx, lw, lb)]

    prev = conv.set_wgrad_overlap(False)
    prev_us = conv.set_fork_min_us(0)  # fork every layer, however small
    try:
        serial = run()
        conv.set_wgrad_overlap(True)
        for _ in range(3):
            got = run()
            assert all(torch.equal(a, c) for a, c in zip(got, serial))
    finally:
        conv.set_wgrad_overlap(prev)
        conv.set_fork_min_us(prev_us)


# k_conv_lp (csrc/conv_lp.hip): the bf16 / fp16 forward and data-gradient kernel, every conv
# geometry of CASES, every block tile (e2ep_tune key 10 = wm * 10 + wn; 1 = automatic), against
# fp64 convolutions of the rounded operands (bias, ReLU and the skip gradient in fp32).
LP_TILES = [1, 11, 12, 14, 21, 22]


@pytest.mark.parametrize("lk", [1, 32, 128], ids=["lkauto", "lk32", "lkw128"])
@pytest.mark.parametrize("tile", LP_TILES, ids=[f"t{t}" for t in LP_TILES])
@pytest.mark.parametrize("case", CASES, ids=[str(i) for i in range(len(CASES))])
def test_conv_lp_kernel_all_geometries(case, tile, lk):
    """lk: K-step depth (e2ep_tune key 16 for k_conv_lp: automatic = 64 channels for 16-bit
    operands, or 32; key 17 for k_wgrad_lp: automatic = 64 pixels, 32 or 128)."""
    from e2ep_amd import _lib, conv, precision
    N, Cin, H, W, Cout, R, S, st, pad, dil, has_b, act = case
    mode, dt = ("fp16", torch.float16) if tile == 12 else ("bf16", torch.bfloat16)
    g = torch.Generator().manual_seed(hash(case) & 0xFFFF)
    x = torch.randn(N, Cin, H, W, generator=g)
    w = torch.randn(Cout, Cin, R, S, generator=g) / (Cin * R * S) ** 0.5
    b = torch.randn(Cout, generator=g) if has_b else None
    if H * W == 1 and R * S == 1:
        pytest.skip("1x1 convs on 1x1 maps run on the fp32 skinny GEMM in every mode")
    xd = x.to(DEV).requires_grad_(True)
    wd = w.to(DEV).requires_grad_(True)
    old_t = _lib.call_raw("e2ep_tune", 10, tile)
    old_lp = _lib.call_raw("e2ep_tune", 11, 2)
    old_wt = _lib.call_raw("e2ep_tune", 13, tile if tile in (11, 12, 21, 22) else 1)
    old_wlp = _lib.call_raw("e2ep_tune", 12, 2)
    old_lk = _lib.call_raw("e2ep_tune", 16, 32 if lk == 32 else 1)
    old_wlk = _lib.call_raw("e2ep_tune", 17, lk)
    try:
        with precision.use(mode):
            y = conv.conv2d(xd, wd, b.to(DEV) if has_b else None, (st, st), pad, (dil, dil), act)
            gy = torch.randn(y.shape, generator=g)
            y.backward(gy.to(DEV))
    finally:
        for k, v in ((10, old_t), (11, old_lp), (13, old_wt), (12, old_wlp), (16, old_lk), (17, old_wlk)):
            _lib.call_raw("e2ep_tune", k, v)
    r = lambda t: t.to(dt).double()  # noqa: E731
    xr = r(x).requires_grad_(True)
    y_r = F.conv2d(F.pad(xr, pad), r(w), b.double() if has_b else None, st, 0, dil)
    if act:
        y_r = torch.relu(y_r)
    # the data gradient takes the gradient through the product's own ReLU mask, rounded
    gy_in = gy.double() * (y.detach().cpu() > 0) if act else gy.double()
    F.conv2d(F.pad(xr, pad), r(w), None, st, 0, dil).backward(r(gy_in.float()))
    if Cin * R * S <= 32 and R * S > 1 and Cout <= 64:
        # the direct forward kernel (k_conv_direct, the EfficientNet stem) is fp32 in every mode
        y64 = F.conv2d(F.pad(x.double(), pad), w.double(), b.double() if has_b else None, st, 0, dil)
        assert rel_l2(y, torch.relu(y64) if act else y64) < 2e-6
    else:
        assert rel_l2(y, y_r) < 2e-6
    assert rel_l2(xd.grad, xr.grad) < 2e-6
    # weight gradient: bf16 operands (x and the gradient at the conv output) in C3 (k_wgrad_lp,
    # key 13 = its tile), fp32 in the fp16 inference mode
    if mode == "bf16":
        wr = r(w).requires_grad_(True)
        F.conv2d(F.pad(r(x), pad), wr, None, st, 0, dil).backward(r(gy_in.float()))
        assert rel_l2(wd.grad, wr.grad) < 5e-6
    else:
        w64 = w.double().requires_grad_(True)
        F.conv2d(F.pad(x.double(), pad), w64, None, st, 0, dil).backward(gy_in)
        assert rel_l2(wd.grad, w64.grad) < 2e-6


@pytest.mark.parametrize("case", SKIP_CASES, ids=[str(i) for i in range(len(SKIP_CASES))])
def test_conv_lp_skip_gradient_fused(case):
    """k_conv_lp data gradient with the skip gradient added in its epilogue / reduction."""
    from e2ep_amd import conv, precision
    N, Cin, H, W, Cout, R, S, pad, gc = case
    g = torch.Generator().manual_seed(17 + Cin)
    x = torch.randn(N, Cin, H, W, generator=g)
    w = torch.randn(Cout, Cin, R, S, generator=g) / (Cin * R * S) ** 0.5
    xd = x.to(DEV).requires_grad_(True)
    wd = w.to(DEV).requires_grad_(True)
    with precision.use("bf16"):
        y, xs = conv.conv2d(xd, wd, None, (1, 1), pad, (1, 1), 0, grad_channels=gc, skip=True)
        gy = torch.randn(y.shape, generator=g)
        gs = torch.randn(x.shape, generator=g)
        ((y * gy.to(DEV)).sum() + (xs * gs.to(DEV)).sum()).backward()
    r = lambda t: t.to(torch.bfloat16).double()  # noqa: E731
    xr = r(x).requires_grad_(True)
    y_r = F.conv2d(F.pad(xr, pad), r(w))
    (y_r * r(gy)).sum().backward()
    gx = xr.grad.clone()
    if gc is not None:
        gx[:, gc:] = 0
    gx += gs.double()
    assert rel_l2(y.detach().cpu(), y_r) < 2e-6
    assert rel_l2(xd.grad.cpu(), gx) < 2e-6


@pytest.mark.parametrize("tile", [1, 11, 12, 21, 22], ids=["t1", "t11", "t12", "t21", "t22"])
@pytest.mark.parametrize("case", CASES, ids=[str(i) for i in range(len(CASES))])
def test_conv_lp_fp32_all_geometries(case, tile):
    """k_conv_lp / k_wgrad_lp with exact-f32 MFMA operands (e2ep_tune keys 14 / 15 = 2), every
    tile (keys 10 / 13), vs fp64: forward, data and weight gradients."""
    from e2ep_amd import _lib, conv
    N, Cin, H, W, Cout, R, S, st, pad, dil, has_b, act = case
    if H * W == 1 and R * S == 1:
        pytest.skip("1x1 convs on 1x1 maps run on the skinny GEMM")
    g = torch.Generator().manual_seed(hash(case) & 0xFFFF)
    x = torch.randn(N, Cin, H, W, generator=g)
    w = torch.randn(Cout, Cin, R, S, generator=g) / (Cin * R * S) ** 0.5
    b = torch.randn(Cout, generator=g) if has_b else None
    xd = x.to(DEV).requires_grad_(True)
    wd = w.to(DEV).requires_grad_(True)
    keys = ((14, 2), (15, 2), (10, tile), (13, tile))
    old = [_lib.call_raw("e2ep_tune", k, v) for k, v in keys]
    try:
        y = conv.conv2d(xd, wd, b.to(DEV) if has_b else None, (st, st), pad, (dil, dil), act)
        gy = torch.randn(y.shape, generator=g)
        y.backward(gy.to(DEV))
    finally:
        for (k, _), v in zip(keys, old):
            _lib.call_raw("e2ep_tune", k, v)
    x64 = x.double().requires_grad_(True)
    w64 = w.double().requires_grad_(True)
    y64 = F.conv2d(F.pad(x64, pad), w64, b.double() if has_b else None, st, 0, dil)
    if act:
        y64 = torch.relu(y64)
    y64.backward(gy.double())
    assert rel_l2(y, y64) < 2e-6
    assert rel_l2(xd.grad, x64.grad) < 2e-6
    assert rel_l2(wd.grad, w64.grad) < 2e-6


@pytest.mark.parametrize("case", CASES + [(2, 160, 8, 8, 960, 1, 1, 1, (0, 0, 0, 0), 1, False, 0),
                                          (8, 256, 16, 16, 256, 3, 3, 1, (1, 1, 1, 1), 1, False, 1),
                                          (8, 512, 8, 8, 512, 3, 3, 1, (1, 1, 1, 1), 1, True, 0)],
                         ids=[str(i) for i in range(len(CASES) + 3)])
@pytest.mark.parametrize("skip", [False, True], ids=["noskip", "skip"])
@pytest.mark.parametrize("mode", ["fp32", "bf16"])
@pytest.mark.parametrize("order", [1, 2], ids=["dgrad_first", "wgrad_first"])  # 1x1 pair order (key 30)
def test_conv_bwd_pair_bitwise_equals_two_launches(case, skip, mode, order):
    """e2ep_conv_bwd (data and weight gradient in one k_conv_bwd_pair / k_lp_bwd_pair launch,
    where e2ep_conv_bwd_pair_ok) == e2ep_conv_dgrad_acc + e2ep_conv_wgrad on forked streams,
    bitwise, with and without the skip gradient added in the data gradient's epilogue; fp32
    (k_conv_gemm or k_conv_lp data gradient) and C3 bf16 operands (k_conv_lp + k_wgrad_lp)."""
    from e2ep_amd import conv, precision
    N, Cin, H, W, Cout, R, S, st, pad, dil, has_b, act = case
    g = torch.Generator().manual_seed(hash(case) & 0xFFFF)
    x = torch.randn(N, Cin, H, W, generator=g).to(DEV)
    w = (torch.randn(Cout, Cin, R, S, generator=g) / (Cin * R * S) ** 0.5).to(DEV)
    b = torch.randn(Cout, generator=g).to(DEV) if has_b else None
    gs = torch.randn(x.shape, generator=g).to(DEV) if skip else None

    def run():
        xd, wd = x.clone().requires_grad_(True), w.clone().requires_grad_(True)
        bd = b.clone().requires_grad_(True) if has_b else None
        out = conv.conv2d(xd, wd, bd, (st, st), pad, (dil, dil), act, skip=skip)
        y = out[0] if skip else out
        gy = torch.randn(y.shape, generator=torch.Generator().manual_seed(5)).to(DEV)
        loss = (y * gy).sum() + ((out[1] * gs).sum() if skip else 0)
        loss.backward()
        return [t.grad.clone() for t in (xd, wd, bd) if t is not None]

    from e2ep_amd import _lib
    lib = _lib.load()
    prev = conv.set_conv_pair(False)
    prev_order1 = lib.e2ep_tune(30, order)  # block order of the paired 1x1 grids
    try:
        with precision.use(mode):
            two = run()
            conv.set_conv_pair(True)
            one = run()
    finally:
        conv.set_conv_pair(prev)
        lib.e2ep_tune(30, prev_order1)
    assert all(torch.equal(a, c) for a, c in zip(one, two))


def test_conv_bwd_pair_covers_small_map_layers():
    """The EfficientNet 1x1 convs on 32x32 and smaller maps and the 16x16 heads' 1x1s take the
    paired backward (their two GEMMs each fill a fraction of the chip) — a plan change that
    drops them back to two forked launches shows up here."""
    from e2ep_amd import _lib
    lib = _lib.load()

    def d1(N, C, H, W, Co):  # (N, Cin, H, W, Cout, R, S, P, Q, sh, sw, pt, pl, dh, dw)
        return (N, C, H, W, Co, 1, 1, H, W, 1, 1, 0, 0, 1, 1)
    layers = [d1(32, 192, 32, 32, 32), d1(32, 336, 16, 16, 56), d1(32, 1152, 8, 8, 192),
              d1(32, 64, 16, 16, 160),
              # 64x64 / 128x128 maps: the k_wgrad_1x1 weight gradient (k_conv_bwd_pair1x1)
              d1(32, 32, 64, 64, 192), d1(32, 192, 64, 64, 32), d1(32, 24, 128, 128, 144)]
    ok = [lib.e2ep_conv_bwd_pair_ok(_lib.dims(d), d[1]) for d in layers]
    assert all(ok), ok
    # BEV encoder / head 3x3s: k_conv_lp data gradient (fp32 and C3 bf16)
    from e2ep_amd import precision
    d3 = [(32, 256, 16, 16, 256, 3, 3, 16, 16, 1, 1, 1, 1, 1, 1),
          (32, 128, 32, 32, 128, 3, 3, 32, 32, 1, 1, 1, 1, 1, 1)]
    for mode in ("fp32", "bf16"):
        with precision.use(mode):
            ok = [lib.e2ep_conv_bwd_pair_ok(_lib.dims(d), d[1]) for d in d3]
        assert all(ok), (mode, ok)
