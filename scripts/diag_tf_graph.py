"""torch TransformerDecoder fwd+bwd captured in a HIP graph vs eager (no e2ep code)."""
import sys

import torch

torch.manual_seed(0)
E, H, L, S, B = 258, 6, 4, 256, 8
blas = sys.argv[1] if len(sys.argv) > 1 else "default"
if blas == "math":
    torch.backends.cuda.enable_flash_sdp(False)
    torch.backends.cuda.enable_mem_efficient_sdp(False)
elif blas != "default":
    torch.backends.cuda.preferred_blas_library(blas)
print("blas:", torch.backends.cuda.preferred_blas_library(), flush=True)
layer = torch.nn.TransformerDecoderLayer(E, H, 2048, dropout=0.0)
dec = torch.nn.TransformerDecoder(layer, L).cuda().train()
mem0 = torch.randn(S, B, E, device="cuda")
tgt0 = torch.randn(14, B, E, device="cuda")
mask = torch.full((14, 14), float("-inf"), device="cuda").triu(1)
pad = torch.zeros(B, 14, dtype=torch.bool, device="cuda")
pad[:, 10:] = True
params = list(dec.parameters())


def step():
    for p in params:
        p.grad = None
    mem = mem0.clone().requires_grad_()
    y = dec(tgt0, mem, tgt_mask=mask, tgt_key_padding_mask=pad, tgt_is_causal=True)
    y.square().mean().backward()
    return mem.grad


ref_mg = step().clone()
ref = [p.grad.clone() for p in params]
s = torch.cuda.Stream()
s.wait_stream(torch.cuda.current_stream())
with torch.cuda.stream(s):
    for _ in range(2):
        step()
torch.cuda.current_stream().wait_stream(s)
g = torch.cuda.CUDAGraph()
with torch.cuda.graph(g):
    junk = torch.empty(1 << 22, device="cuda")
    junk.fill_(3.0e38)
    del junk
    mg = step()
for r in range(2):
    g.replay()
    torch.cuda.synchronize()
    names = [n for n, _ in dec.named_parameters()]
    bad = [(n, float((p.grad - q).norm() / (q.norm() + 1e-30))) for n, p, q in zip(names, params, ref)]
    bad = [b for b in bad if not b[1] < 1e-5]
    print("replay", r, "mem grad rel", float((mg - ref_mg).norm() / ref_mg.norm()),
          "param mismatches", len(bad), bad[:6], flush=True)
