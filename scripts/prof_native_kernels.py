"""Diagnostics: every PyTorch-native (at::native) GPU kernel one eager TrainStep (the bench's
step: fwd + 3 losses + bwd + Adam, B = 8) launches, with the aten op that launched it and the
model / product source line of that op.

    python scripts/prof_native_kernels.py [--precision bf16] > gpurun_out/native_kernels.txt"""
import argparse
import collections
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "e2e-parking-carla_amd"), ROOT]
import torch  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--precision", default="fp32")
    a = ap.parse_args()
    from bench import device_batch
    from e2ep_amd import precision, synthetic
    from e2ep_amd.train import TrainStep
    from tool.config import default_cfg
    from trainer.pl_trainer import ParkingTrainingModule

    precision.set(a.precision)
    dev = torch.device("cuda")
    torch.manual_seed(1234)
    mod = ParkingTrainingModule(default_cfg()).to(dev).train()
    for p in mod.parking_model.bev_encoder.layer4.parameters():
        p.requires_grad_(False)
    data = device_batch(synthetic.synthetic_batch(8, seed=0), dev)
    step = TrainStep(mod, data, lr=mod.cfg.learning_rate, weight_decay=mod.cfg.weight_decay,
                     world=1, graph=False, warmup=1)
    for _ in range(2):
        step()
    torch.cuda.synchronize()
    # every aten op that can launch a kernel, with the autograd node executing it (backward)
    # or the first product source frame (forward)
    import traceback
    from torch.utils._python_dispatch import TorchDispatchMode
    skip = ("empty", "view", "as_strided", "reshape", "detach", "t", "transpose", "expand",
            "_unsafe_view", "slice", "select", "unsqueeze", "squeeze", "permute", "alias",
            "empty_like", "empty_strided", "lift_fresh", "resolve_conj", "resolve_neg", "item",
            "_local_scalar_dense", "is_nonzero", "narrow", "split", "chunk", "unbind", "split_with_sizes",
            "new_empty", "new_empty_strided", "clone_if_view", "set_", "result_type", "size",
            "stride", "numel", "dim", "is_contiguous", "contiguous", "_to_copy", "to", "_reshape_alias",
            "sym_size", "sym_stride", "sym_numel", "sym_storage_offset", "storage_offset", "zeros_like")
    keys = ("model/", "e2ep_amd/", "loss/", "trainer/", "bench.py")
    rows = collections.Counter()

    class Log(TorchDispatchMode):
        def __torch_dispatch__(self, func, types, args=(), kwargs=None):
            out = func(*args, **(kwargs or {}))
            name = func.overloadpacket.__name__
            tens = [t for t in torch.utils._pytree.tree_leaves((args, kwargs, out))
                    if isinstance(t, torch.Tensor)]
            if name in skip or not any(t.is_cuda for t in tens) or all(t.numel() == 0 for t in tens):
                return out
            node = torch._C._current_autograd_node()
            if node is not None:
                site = "backward of " + node.name()
                if name in ("add", "add_"):  # which input buffer: the node's next functions
                    nxt = [f.name() for f, _ in node.next_functions if f is not None]
                    site += " -> " + ",".join(nxt[:4])
            else:
                fr = [f for f in traceback.extract_stack() if any(k in f.filename for k in keys)]
                site = f"{fr[-1].filename.split('/root/repo/')[-1]}:{fr[-1].lineno} {fr[-1].name}" if fr else "(no product frame)"
            shp = [tuple(t.shape) for t in tens][:2]
            rows[(str(func), site, str(shp))] += 1
            return out

    with Log():
        step()
        torch.cuda.synchronize()
    for (fn, site, shp), n in sorted(rows.items(), key=lambda r: (-r[1], r[0])):
        print(f"{n:4d}  {fn:40s} {site}  {shp}")
    print(f"total aten ops on the device: {sum(rows.values())}")


if __name__ == "__main__":
    main()
