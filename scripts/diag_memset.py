"""Are zero-fills (hipMemsetAsync) inside a captured HIP graph replayed?"""
import torch

x = torch.ones(1 << 20, device="cuda")
for n in (1, 3, 64, 258, 516, 774, 1000, 4096, 65536, 1 << 20):
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        z = torch.zeros(n, device="cuda")
        z += x[:n]
    res = []
    for r in range(3):
        g.replay()
        torch.cuda.synchronize()
        res.append(float(z.max()))
    print(n, "max after replays (want 1.0):", res, flush=True)
