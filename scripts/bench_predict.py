"""C5 (BASELINE.json configs[4]): closed-loop inference latency of ParkingModel.predict at
B=1 — the call agent/parking_agent.py:385 makes every control step (encoder + 3
autoregressive ControlPredict passes, reference model/parking_model.py:72-78).

    python scripts/bench_predict.py [--iters 200] [--cpu-iters 5] [--precision fp16] [--json out.json]
Reports p50/p90 latency (ms) of (a) eager predict and (b) predict captured once into a HIP
graph and replayed (static input buffers; the per-call inputs are copied into them on the
stream, included in the timing), each call synchronised, plus the oracle (CPU restatement of
the reference) on the host cores.  --precision fp16 (C5) runs the conv GEMMs on fp16 operands
(fp32 accumulation; e2ep_amd.precision); the tokens are compared with the fp32 run's."""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "e2e-parking-carla_amd"), ROOT]
import numpy as np  # noqa: E402
import torch  # noqa: E402


def pct(ts, q):
    return float(np.percentile(np.asarray(ts) * 1e3, q))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--iters", type=int, default=200)
    ap.add_argument("--cpu-iters", type=int, default=5)
    ap.add_argument("--json", default=None)
    ap.add_argument("--precision", choices=("fp32", "fp16", "bf16"), default="fp32")
    a = ap.parse_args()
    from e2ep_amd import _lib, graphs, precision, synthetic
    from model.parking_model import ParkingModel
    from tool.config import default_cfg

    _lib.load()
    dev = torch.device("cuda")
    torch.manual_seed(0)
    m = ParkingModel(default_cfg()).to(dev).eval()
    host = synthetic.synthetic_batch(1, seed=0)
    host["gt_control"] = host["gt_control"][:, :1]  # BOS: the agent's first token
    keys = ("image", "target_point", "ego_motion", "gt_control")
    static = {k: host[k].to(dev) for k in keys}
    static["intrinsics"], static["extrinsics"] = host["intrinsics"], host["extrinsics"]

    noise = synthetic.target_noise(1, seed=0).to(dev)  # fixed target jitter: comparable tokens

    def call():
        with torch.no_grad():
            return m.predict(static, noise)

    with torch.no_grad():  # fp32 tokens, for the low-precision comparison
        ref_tokens = m.predict(static, noise)[0].clone()
    precision.set(a.precision)

    # (a) eager
    for _ in range(5):
        call()
    torch.cuda.synchronize()
    eager = []
    for _ in range(a.iters):
        t0 = time.perf_counter()
        for k in keys:
            static[k].copy_(host[k], non_blocking=True)
        out = call()
        torch.cuda.synchronize()
        eager.append(time.perf_counter() - t0)

    # (b) HIP graph: capture on a side stream after warm-up, replay
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        for _ in range(3):
            call()
    torch.cuda.current_stream().wait_stream(s)
    torch.cuda.synchronize()
    g, gout, nmem = graphs.capture(call)
    graph = []
    for _ in range(a.iters):
        t0 = time.perf_counter()
        for k in keys:
            static[k].copy_(host[k], non_blocking=True)
        g.replay()
        torch.cuda.synchronize()
        graph.append(time.perf_counter() - t0)
    same = bool(torch.equal(gout[0], out[0]))
    same_fp32 = bool(torch.equal(gout[0], ref_tokens))
    precision.set("fp32")

    # (c) the oracle on the host cores
    cpu = []
    if a.cpu_iters > 0:
        from oracle import parking_ref as O
        torch.set_num_threads(min(16, os.cpu_count() or 1))
        ref = O.ParkingModelRef(O.Cfg).eval()
        with torch.no_grad():
            ref.predict(host)
            for _ in range(a.cpu_iters):
                t0 = time.perf_counter()
                ref.predict(host)
                cpu.append(time.perf_counter() - t0)
    res = {"config": f"C5: ParkingModel.predict, B=1, 4 cams 256x256, conv GEMM operands {a.precision}",
           "precision": a.precision, "iters": a.iters,
           "eager_p50_ms": round(pct(eager, 50), 3), "eager_p90_ms": round(pct(eager, 90), 3),
           "graph_p50_ms": round(pct(graph, 50), 3), "graph_p90_ms": round(pct(graph, 90), 3),
           "graph_tokens_equal_eager": same, "tokens_equal_fp32": same_fp32,
           "tokens": gout[0].cpu().tolist(), "graph_memset_nodes_rewritten": nmem,
           "cpu_oracle_p50_ms": round(pct(cpu, 50), 1) if cpu else None,
           "cpu_threads": torch.get_num_threads() if cpu else None,
           "published_ait_ms_rtx5000": 74.92}
    print(json.dumps(res))
    if a.json:
        json.dump(res, open(a.json, "w"), indent=1)


if __name__ == "__main__":
    main()
