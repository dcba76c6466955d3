"""Per-node cost of a captured HIP graph on this stack: replay time of a chain of N tiny
kernels (1-element in-place add) vs N, on one stream and split over two streams."""
import torch

x = torch.zeros(1, device="cuda")
y = torch.zeros(1, device="cuda")


def timed(g, reps=20):
    g.replay()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(reps):
        g.replay()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / reps


for n in (100, 500, 1000, 2000):
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        for _ in range(n):
            x.add_(1.0)
    ms = timed(g)
    print(f"chain of {n:5d} tiny kernels: {ms:.3f} ms/replay = {1e3 * ms / n:.2f} us/node", flush=True)
side = torch.cuda.Stream()
for n in (1000,):
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        cur = torch.cuda.current_stream()
        side.wait_stream(cur)
        for _ in range(n // 2):
            x.add_(1.0)
        with torch.cuda.stream(side):
            for _ in range(n // 2):
                y.add_(1.0)
        cur.wait_stream(side)
    ms = timed(g)
    print(f"two chains of {n // 2} tiny kernels: {ms:.3f} ms/replay = {1e3 * ms / n:.2f} us/node", flush=True)
