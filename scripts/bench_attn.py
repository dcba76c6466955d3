"""Microbench of the fused attention core on the transformer's three shapes (B = 8, 6 heads x
43): forward and backward kernel time by HIP events over 50 back-to-back launches."""
import sys
import os
import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "e2e-parking-carla_amd"))
from e2ep_amd import attention  # noqa: E402

B, H, E = 8, 6, 258
for name, Sq, Sk, causal in [("enc_self", 256, 256, False), ("dec_self", 14, 14, True),
                             ("dec_cross", 14, 256, False)]:
    packed = name != "dec_cross"
    qb = torch.randn(Sq, B, 3 * E if packed else E, device="cuda", requires_grad=True)
    kvb = None if packed else torch.randn(Sk, B, 2 * E, device="cuda", requires_grad=True)
    seed = torch.tensor([1], dtype=torch.int32, device="cuda")
    o = attention.attention(qb, kvb, H, causal, None, 0.1, seed)
    do = torch.randn_like(o)
    res = {}
    for part in ("fwd", "fwd+bwd"):
        def run():
            o = attention.attention(qb, kvb, H, causal, None, 0.1, seed)
            if part != "fwd":
                torch.autograd.grad(o, [qb] if packed else [qb, kvb], do)
        for _ in range(3):
            run()
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        torch.cuda.synchronize()
        a.record()
        for _ in range(50):
            run()
        b.record()
        torch.cuda.synchronize()
        res[part] = a.elapsed_time(b) / 50 * 1e3
    print(f"{name}: fwd {res['fwd']:.1f} us, fwd+bwd {res['fwd+bwd']:.1f} us (incl. host launch)")
