"""Linear bias-grad under graph replay: which formulation breaks, and how."""
import torch
import torch.nn.functional as F

torch.manual_seed(0)
E = 258
x0 = torch.randn(2048, E, device="cuda")
W2 = torch.randn(516, E, device="cuda") * 0.05
bl = torch.zeros(516, device="cuda").requires_grad_()


def run(name, fn, params):
    out = {}

    def step():
        for p in params:
            p.grad = None
        fn().square().mean().backward()
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
    res = []
    for r in range(3):
        g.replay()
        torch.cuda.synchronize()
        a, c = out["g"][0], ref[0]
        res.append("err %.1e ratio[min %.4f max %.4f]" % (float((a - c).norm() / c.norm()),
                                                         float((a / c).min()), float((a / c).max())))
    print(f"{name:22s}", res, flush=True)


run("addmm bias only", lambda: F.linear(x0, W2, bl), [bl])
Wg = W2.clone().requires_grad_()
run("addmm bias+weight", lambda: F.linear(x0, Wg, bl), [bl, Wg])
xg = x0.clone().requires_grad_()
run("addmm bias+input", lambda: F.linear(xg, W2, bl), [bl, xg])
run("mm + add", lambda: x0 @ W2.t() + bl, [bl])
run("bias broadcast only", lambda: x0[:, :1] * 0.5 + bl, [bl])
run("sum(0) of grad-like", lambda: (x0 @ W2.t()).detach() * 0 + bl * x0[:, :516], [bl])
