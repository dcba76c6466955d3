"""Which torch reductions go wrong when replayed from a HIP graph (inputs change per replay)?"""
import torch
import torch.nn.functional as F

torch.manual_seed(0)
W = torch.tensor([1.0, 2.0, 3.0], device="cuda")
cases = {
    "sum0_2048x516": ((2048, 516), lambda x: x.sum(0)),
    "sum01_256x8x516": ((256, 8, 516), lambda x: x.sum((0, 1))),
    "sum01_perm": ((8, 256, 516), lambda x: x.transpose(0, 1).sum((0, 1))),
    "sum0_14x8x258": ((14, 8, 258), lambda x: x.sum((0, 1))),
    "sum_all_3M": ((3_200_000,), lambda x: x.sum()),
    "mean_rows_65536x8": ((65536, 8), lambda x: x.mean(0)),
    "ce_w_ign": ((8, 3, 200, 200), lambda x: F.cross_entropy(
        x, (x[:, 0] * 7).long().abs() % 4, weight=W, ignore_index=3)),
    "bce": ((8, 48, 32, 32), lambda x: F.binary_cross_entropy(x.sigmoid(), (x > 0).float())),
    "norm": ((1 << 20,), lambda x: x.norm()),
    "var_mean": ((64, 4096), lambda x: torch.var_mean(x, 1)[0]),
}
for name, (shape, fn) in cases.items():
    x = torch.randn(*shape, device="cuda")
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        fn(x)
    torch.cuda.current_stream().wait_stream(s)
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        y = fn(x)
    errs = []
    for r in range(4):
        x.copy_(torch.randn(*shape, device="cuda"))
        g.replay()
        torch.cuda.synchronize()
        ref = fn(x)
        errs.append(float(((y - ref).abs().max() / (ref.abs().max() + 1e-30))))
    print(f"{name:20s}", ["%.1e" % e for e in errs], flush=True)
