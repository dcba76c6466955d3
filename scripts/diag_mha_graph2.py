"""Narrow the graph-replay gradient bug: backward() vs autograd.grad, slice vs leaf bias."""
import torch
import torch.nn.functional as F

torch.manual_seed(0)
E, H, S, T, B = 258, 6, 256, 14, 8
mha = torch.nn.MultiheadAttention(E, H).cuda()
q0 = torch.randn(T, B, E, device="cuda")
m0 = torch.randn(S, B, E, device="cuda")
w, b = mha.in_proj_weight, mha.in_proj_bias
bleaf = b[E:].detach().clone().requires_grad_()
W2 = w[E:].detach().clone()


def run(name, fn, params, use_grad):
    out = {}

    def step():
        for p in params:
            p.grad = None
        loss = fn().square().mean()
        if use_grad:
            gs = torch.autograd.grad(loss, params)
            out["g"] = gs
        else:
            loss.backward()
            out["g"] = [p.grad for p in params]
    step()
    ref = [g.clone() for g in out["g"]]
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
        errs.append(max(float((a - c).norm() / c.norm()) for a, c in zip(out["g"], ref)))
    print(f"{name:28s}", ["%.1e" % e for e in errs], flush=True)


cross = lambda: mha(q0, m0, m0, need_weights=False)[0]
run("cross backward", cross, [w, b], False)
run("cross autograd.grad", cross, [w, b], True)
run("linear slice-bias backward", lambda: F.linear(m0, W2, b[E:]), [b], False)
run("linear slice-bias grad", lambda: F.linear(m0, W2, b[E:]), [b], True)
run("linear leaf-bias backward", lambda: F.linear(m0, W2, bleaf), [bleaf], False)
run("linear 2d leaf-bias backward", lambda: F.linear(m0.reshape(-1, E), W2, bleaf), [bleaf], False)
run("sum-only leaf", lambda: (m0[..., :1] * 0 + bleaf), [bleaf], False)
