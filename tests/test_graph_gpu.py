"""Captured HIP graphs replay correctly after the memset-node repair (e2ep_amd.graphs).

Without the repair, a hipMemsetAsync captured into a graph leaves garbage from the second
replay on, and PyTorch's captured reductions (bias gradients of broadcast adds) go wrong
(one-off diagnostics, git history at cb07871^)."""
import ctypes

import pytest
import torch

pytestmark = pytest.mark.gpu


def _hip():
    hip = ctypes.CDLL("libamdhip64.so")
    hip.hipMemsetAsync.argtypes = [ctypes.c_void_p, ctypes.c_int, ctypes.c_size_t, ctypes.c_void_p]
    return hip


@pytest.mark.parametrize("nbytes", [4, 100, 4096, 1 << 20])
def test_repaired_memset_node_replays(nbytes):
    from e2ep_amd import graphs
    hip = _hip()
    buf = torch.full((nbytes,), 7, dtype=torch.uint8, device="cuda")

    def body():
        hip.hipMemsetAsync(ctypes.c_void_p(buf.data_ptr()), 0, nbytes,
                           ctypes.c_void_p(torch.cuda.current_stream().cuda_stream))
        buf.add_(1)
    g, _, n = graphs.capture(body)
    assert n == 1
    for _ in range(4):
        g.replay()
        torch.cuda.synchronize()
        assert int(buf.min()) == 1 and int(buf.max()) == 1


def test_captured_bias_grad_replays():
    from e2ep_amd import graphs
    torch.manual_seed(0)
    x = torch.randn(2048, 258, device="cuda")
    b = torch.zeros(516, device="cuda", requires_grad=True)
    out = {}

    def step():
        b.grad = None
        (x[:, :1] * 0.5 + b).square().mean().backward()
        out["g"] = b.grad
    step()
    ref = b.grad.clone()
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        step()
    torch.cuda.current_stream().wait_stream(s)
    g, _, _ = graphs.capture(step)
    for _ in range(4):
        g.replay()
        torch.cuda.synchronize()
        assert torch.allclose(out["g"], ref, rtol=1e-6, atol=1e-9)


def test_captured_predict_matches_eager():
    """C5 path: ParkingModel.predict (B=1, eval) captured into one HIP graph replays the eager
    result — control tokens identical, segmentation / depth bitwise equal (fixed noise)."""
    from e2ep_amd import graphs, synthetic
    from model.parking_model import ParkingModel
    from tool.config import default_cfg
    torch.manual_seed(0)
    m = ParkingModel(default_cfg()).cuda().eval()
    host = synthetic.synthetic_batch(1, seed=2)
    host["gt_control"] = host["gt_control"][:, :1]
    data = {k: (v if k in ("intrinsics", "extrinsics") else v.cuda()) for k, v in host.items()}
    noise = synthetic.target_noise(1, seed=2).cuda()

    def call():
        with torch.no_grad():
            return m.predict(data, noise)
    ref = call()
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        call()
    torch.cuda.current_stream().wait_stream(s)
    g, out, _ = graphs.capture(call)
    for _ in range(3):
        g.replay()
        torch.cuda.synchronize()
        assert torch.equal(out[0], ref[0])
        assert torch.equal(out[1], ref[1]) and torch.equal(out[2], ref[2])
        assert torch.equal(out[3], ref[3])


def test_torch_rng_in_capture_draws_fresh_values_per_replay():
    """A capture that draws from torch's generators (a user module's dropout, rng.py's torch
    fallback outside a step pool) replays through torch's replay, whose prologue advances the
    generator offsets: every replay draws new values, as eager calls would.  A
    capture without such draws keeps the owned executable."""
    from e2ep_amd import graphs, rng
    rng.end_step()  # no step pool: rng.uniform / rng.seed fall back to torch draws
    u = torch.empty(4096, device="cuda")
    m = torch.empty(4096, device="cuda")
    s = torch.empty(1, dtype=torch.int32, device="cuda")
    ones = torch.ones(4096, device="cuda")

    def body():
        u.copy_(rng.uniform((4096,), "cuda"))
        m.copy_(torch.nn.functional.dropout(ones, 0.5, training=True))
        s.copy_(rng.seed("cuda"))
    g, _, _ = graphs.capture(body)
    assert g.torch_rng and g._exec is None
    seen = []
    for _ in range(3):
        g.replay()
        torch.cuda.synchronize()
        seen.append((u.clone(), m.clone(), int(s)))
    for a, b in zip(seen, seen[1:]):
        assert not torch.equal(a[0], b[0]) and not torch.equal(a[1], b[1]) and a[2] != b[2]
    assert all(0.0 <= float(t[0].min()) and float(t[0].max()) < 1.0 for t in seen)

    buf = torch.zeros(16, device="cuda")
    g2, _, _ = graphs.capture(lambda: buf.add_(1))
    assert not g2.torch_rng and g2._exec is not None
    g2.replay()
    g2.replay()
    torch.cuda.synchronize()
    assert float(buf[0]) == 2.0


def test_capture_raises_on_unjoined_side_stream():
    """graphs.capture checks, before the capture ends, that every side stream forked into it
    (model branches, weight-gradient forks) rejoined the capturing stream
    (e2ep_capture_unjoined): a fork left open raises E2EPError naming the stream (joined
    first, so the capture still ends cleanly) instead of reaching hipStreamEndCapture; a
    joined fork captures and replays."""
    from e2ep_amd import _lib, conv, graphs
    dev = torch.device("cuda", torch.cuda.current_device())
    buf = torch.zeros(1024, device="cuda")

    def body(join):
        def f():
            with conv._Fork(dev) as side:
                buf.add_(1)
            if join:
                side.join()
            buf.mul_(2)
        return f
    g, _, _ = graphs.capture(body(True))
    g.replay()
    torch.cuda.synchronize()
    assert float(buf[0]) == 2.0
    with pytest.raises(_lib.E2EPError, match="never rejoined"):
        graphs.capture(body(False))
    torch.cuda.synchronize()
