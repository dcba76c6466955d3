"""Isolate the torch op whose gradient goes wrong on the 2nd replay of a captured graph."""
import torch
import torch.nn.functional as F

torch.manual_seed(0)
E, H, S, T, B = 258, 6, 256, 14, 8
mha = torch.nn.MultiheadAttention(E, H).cuda()
q0 = torch.randn(T, B, E, device="cuda")
m0 = torch.randn(S, B, E, device="cuda")
w, b = mha.in_proj_weight, mha.in_proj_bias


def v_cross():
    mem = m0.clone().requires_grad_()
    return mha(q0, mem, mem, need_weights=False)[0]


def v_cross_sep():
    mem = m0.clone().requires_grad_()
    return mha(q0, mem, mem.clone(), need_weights=False)[0]


def v_self():
    return mha(q0, q0, q0, need_weights=False)[0]


def v_kvproj():
    _, w_kv = w.split([E, 2 * E])
    _, b_kv = b.split([E, 2 * E])
    return F.linear(m0, w_kv, b_kv)


def v_kvproj_unflat():
    _, w_kv = w.split([E, 2 * E])
    _, b_kv = b.split([E, 2 * E])
    kv = F.linear(m0, w_kv, b_kv)
    kv = kv.unflatten(-1, (2, E)).unsqueeze(0).transpose(0, -2).squeeze(-2).contiguous()
    return kv[0] * kv[1]


def v_linear_only():
    return F.linear(m0, w[E:].detach(), b[E:])


for name, fn in [("cross", v_cross), ("cross_sep", v_cross_sep), ("self", v_self),
                 ("kvproj", v_kvproj), ("kvproj_unflat", v_kvproj_unflat), ("linear_only", v_linear_only)]:
    def step():
        mha.zero_grad(set_to_none=True)
        fn().square().mean().backward()
    step()
    ref = b.grad.clone()
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        step()
    torch.cuda.current_stream().wait_stream(s)
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        step()
    errs = []
    for r in range(3):
        g.replay()
        torch.cuda.synchronize()
        errs.append(float((b.grad - ref).norm() / ref.norm()))
    print(f"{name:14s} in_proj_bias grad rel err per replay:", ["%.1e" % e for e in errs], flush=True)
