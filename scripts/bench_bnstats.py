"""Cost of the BatchNorm statistics epilogue (e2ep_conv_fwd_stats / e2ep_dwconv_fwd_stats)
against the plain forward and the k_bn_stats pass it replaces, per C2 split-path BN layer shape
(EfficientNet expand / project 1x1 convs and depthwise convs with N*H*W > 8192), in isolation:
mean of 20 back-to-back launches, HIP events on the launch stream.

    python scripts/bench_bnstats.py
"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "e2e-parking-carla_amd"), ROOT]


def timed(fn, iters=20):
    import torch
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(iters):
        fn()
    e.record()
    torch.cuda.synchronize()
    return 1000.0 * s.elapsed_time(e) / iters


def main():
    import torch
    from e2ep_amd import _lib, conv
    lib = _lib.load()
    dev = "cuda"
    # (N, Cin, H, W, Cout): MBConv 1x1 convs whose BN takes the split path at C2 (N = 32)
    convs = [(32, 24, 128, 128, 144), (32, 144, 64, 64, 32), (32, 32, 64, 64, 192),
             (32, 192, 64, 64, 32), (32, 192, 32, 32, 56), (32, 56, 32, 32, 336),
             (32, 336, 32, 32, 56)]
    print("conv 1x1 (N, Cin, H, W, Cout): plain / +stats / k_bn_stats+finalize -> finalize from partials (us)")
    for N, Cin, H, W, Cout in convs:
        dims = (N, Cin, H, W, Cout, 1, 1, H, W, 1, 1, 0, 0, 1, 1)
        d = _lib.dims(dims)
        x = torch.randn(N, Cin, H, W, device=dev)
        w = torch.randn(1, Cout, Cin, device=dev)
        y = torch.empty(N, Cout, H, W, device=dev)
        ws = torch.empty(max(16, lib.e2ep_conv_fwd_workspace(d)), dtype=torch.uint8, device=dev)
        tiles = lib.e2ep_conv_fwd_stats_tiles(d, 1)
        st = torch.empty(max(1, Cout * tiles * 2), dtype=torch.float64, device=dev)
        plain = timed(lambda: conv.conv_fwd(x, w, None, dims, 0, y, w_layout=1))
        withs = timed(lambda: conv.conv_fwd(x, w, None, dims, 0, y, w_layout=1, stats=st)) if tiles else 0.0
        f32 = dict(dtype=torch.float32, device=dev)
        g, b = torch.ones(Cout, **f32), torch.zeros(Cout, **f32)
        out = torch.empty(4, Cout, **f32)
        bws = torch.empty(lib.e2ep_bn_workspace(N, Cout, H, W), dtype=torch.uint8, device=dev)

        def bn_stats():
            _lib.call("e2ep_bn_stats", _lib.ptr(y), _lib.ptr(g), _lib.ptr(b), None, None, N, Cout, H, W,
                      1, 0.1, 1e-3, _lib.ptr(out[0]), _lib.ptr(out[1]), _lib.ptr(out[2]),
                      _lib.ptr(out[3]), _lib.ptr(bws), _lib.nbytes(bws), _lib.stream(), 0)
        bst = timed(bn_stats)
        fin = 0.0
        if tiles:
            def finalize():
                _lib.call("e2ep_bn_finalize_part", _lib.ptr(st), tiles, _lib.ptr(g), _lib.ptr(b), None,
                          None, N, Cout, H, W, 0.1, 1e-3, _lib.ptr(out[0]), _lib.ptr(out[1]),
                          _lib.ptr(out[2]), _lib.ptr(out[3]), None, 0, _lib.stream())
            fin = timed(finalize)
        print(f"  {(N, Cin, H, W, Cout)}: {plain:7.1f} / {withs:7.1f} ({withs - plain:+6.1f}) / "
              f"{bst:7.1f} -> finalize_part {fin:5.1f}   tiles {tiles}")
    # depthwise (N, C, H, W, K, stride, pad l r t b)
    dws = [(32, 144, 128, 128, 3, 2, (0, 1, 0, 1)), (32, 192, 64, 64, 5, 1, (2, 2, 2, 2)),
           (32, 192, 64, 64, 5, 2, (1, 2, 1, 2)), (32, 336, 32, 32, 3, 1, (1, 1, 1, 1))]
    print("depthwise (N, C, H, W, K, s): plain / +stats (us)")
    for N, C, H, W, K, st_, pad in dws:
        l, r, t, b_ = pad
        P = (H + t + b_ - K) // st_ + 1
        Q = (W + l + r - K) // st_ + 1
        dims = (N, C, H, W, K, P, Q, st_, t, l)
        d = _lib.dims(dims)
        x = torch.randn(N, C, H, W, device=dev)
        w = torch.randn(C, 1, K, K, device=dev)
        y = torch.empty(N, C, P, Q, device=dev)
        tiles = lib.e2ep_dwconv_fwd_stats_tiles(d)
        st = torch.empty(max(1, C * tiles * 2), dtype=torch.float64, device=dev)

        def run(stats):
            _lib.call("e2ep_dwconv_fwd_stats", _lib.ptr(x), _lib.ptr(w), d, None, None, 0, _lib.ptr(y),
                      _lib.ptr(stats), _lib.nbytes(stats) if stats is not None else 0, _lib.stream(), 0)
        plain = timed(lambda: run(None))
        withs = timed(lambda: run(st)) if tiles else 0.0
        print(f"  {(N, C, H, W, K, st_)}: {plain:7.1f} / {withs:7.1f} ({withs - plain:+6.1f})  tiles {tiles}")


if __name__ == "__main__":
    main()
