"""Diagnostic: which side-stream branch captures crash hipStreamEndCapture (round 2 and round 4
both saw a segfault in torch.cuda.graph's capture_end with model branches on side streams).

    python scripts/diag_branch_capture.py            # runs every variant in a subprocess
    python scripts/diag_branch_capture.py VARIANT    # one variant in this process

Variants (forward on two streams, loss.backward(), all inside one graph capture, then one
replay compared with eager):
  toy_plain     torch ops: branch on a side stream, joined with wait_stream
  toy_record    the same, plus record_stream on the tensors crossing the streams
  toy_e2ep      the branch made of e2ep conv2d (whose backward forks its weight gradient)
  toy_keep      toy_e2ep captured through e2ep_amd.graphs.capture (keep_graph=True, own exec)
  model_cam     the ParkingModel B=2 train step with streams branch "cam" only
  model_heads   the same with branch "heads" only
  *_nofork      a model variant with the conv weight-gradient side streams off (no stream
                forked from inside a branch)
Round 5: model_cam crashed (exit -11 in capture_end) and model_cam_nofork / model_heads_nofork
replayed, so the crash needs a stream forked from a branch stream; conv._Fork no longer forks
from a branch stream, and model_cam / model_heads are expected to replay too
(profiles/r05/diag_branch_capture*.log).
Round 6: with E2EP_FORK_FROM_BRANCH=1 the nested fork is allowed again, and graphs.capture's
join check (e2ep_capture_unjoined) reports any stream left unjoined before the capture ends.
"""
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "e2e-parking-carla_amd"), ROOT, os.path.join(ROOT, "tests")]
VARIANTS = os.environ.get("DIAG_VARIANTS", "model_cam,model_heads,model_cam_nofork,model_heads_nofork").split(",")


def toy(kind):
    import torch
    from e2ep_amd import conv
    dev = torch.device("cuda")
    torch.manual_seed(0)
    w1 = torch.randn(16, 16, 3, 3, device=dev, requires_grad=True)
    w2 = torch.randn(16, 16, 3, 3, device=dev, requires_grad=True)
    x = torch.randn(4, 16, 32, 32, device=dev)
    side = torch.cuda.Stream()

    def step():
        main = torch.cuda.current_stream()
        side.wait_stream(main)
        if kind == "toy_record":
            x.record_stream(side)
        with torch.cuda.stream(side):
            if kind in ("toy_e2ep", "toy_keep"):
                b = conv.conv2d(x, w2, pad=(1, 1, 1, 1))
            else:
                b = torch.nn.functional.conv2d(x, w2, padding=1)
        a = conv.conv2d(x, w1, pad=(1, 1, 1, 1)) if kind in ("toy_e2ep", "toy_keep") else \
            torch.nn.functional.conv2d(x, w1, padding=1)
        main.wait_stream(side)
        if kind == "toy_record":
            b.record_stream(main)
        loss = (a * b).square().mean()
        w1.grad = w2.grad = None
        loss.backward()
        return loss.detach()

    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        for _ in range(2):
            step()
    torch.cuda.current_stream().wait_stream(s)
    torch.cuda.synchronize()
    eager = step(), w1.grad.clone(), w2.grad.clone()
    if kind == "toy_keep":  # the product's capture: keep_graph=True, memset repair, own exec
        from e2ep_amd import graphs
        g, out, _ = graphs.capture(step)
    else:
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g):
            out = step()
    g.replay()
    torch.cuda.synchronize()
    same = torch.equal(out, eager[0]) and torch.equal(w1.grad, eager[1]) and torch.equal(w2.grad, eager[2])
    print(f"{kind}: captured and replayed; equal to eager: {same}", flush=True)


def model(kind):
    import torch
    from e2ep_amd import conv, streams, synthetic
    from e2ep_amd.train import TrainStep
    from test_train_step_b8_gpu import _module
    if kind.endswith("_nofork"):  # no nested weight-gradient side streams inside the branch
        conv.set_wgrad_overlap(False)
        kind = kind[:-len("_nofork")]
    streams.set_enabled({"model_cam": ["cam"], "model_heads": ["heads"]}[kind])
    mod = _module()
    d = synthetic.synthetic_batch(8, seed=11)
    batch = {k: (v if k in ("intrinsics", "extrinsics") else v.cuda()) for k, v in d.items()}
    step = TrainStep(mod, batch, graph=True, warmup=2)
    losses = [float(step()) for _ in range(3)]
    torch.cuda.synchronize()
    print(f"{kind}: captured and replayed, losses {losses}", flush=True)


def main():
    if len(sys.argv) > 1:
        kind = sys.argv[1]
        (toy if kind.startswith("toy") else model)(kind)
        return
    for kind in VARIANTS:
        env = dict(os.environ, AMD_LOG_LEVEL="1")  # HIP runtime errors on stderr
        r = subprocess.run([sys.executable, "-X", "faulthandler", "-u", __file__, kind],
                           capture_output=True, text=True, timeout=300, env=env)
        tail = (r.stdout.strip().splitlines() or [""])[-1]
        print(f"{kind}: exit {r.returncode} {tail if r.returncode == 0 else ''}", flush=True)
        if r.returncode != 0:
            for ln in r.stderr.splitlines()[-40:]:  # faulthandler's Python stack + HIP errors
                print("   ", ln[:200], flush=True)


if __name__ == "__main__":
    main()
