"""A/B of the BEV stem forward, data gradient and (bf16) weight gradient (conv 7x7/2, 65 -> 64, 256^2 -> 128^2, B = 8) on
16-bit operands: k_conv_stem_lp / k_conv_stem_dgrad_lp / k_conv_stem_wgrad_lp (e2ep_tune key 35 = 1 + mask,
csrc/conv_stem.hip) against the implicit GEMMs k_conv_lp / k_wgrad_lp (key 35 = 1); the weight
gradient's time includes its split reduction.  Mean device time per
call over --iters calls (HIP events; the weight-image prep launch included), after warmup.

    python scripts/bench_stem.py [--mode bf16|fp16|fp32] [--batch 8] [--iters 50]
(fp32: the exact-f32 MFMA variants, key 35 mask 16 / 8, against k_conv_gemm2 / k_conv_wgrad2)"""
import argparse
import json
import os
import sys

import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))),
                                "e2e-parking-carla_amd"))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--mode", default="bf16")
    ap.add_argument("--batch", type=int, default=8)
    ap.add_argument("--iters", type=int, default=50)
    a = ap.parse_args()
    from e2ep_amd import _lib, conv, precision
    g = torch.Generator().manual_seed(0)
    x = torch.randn(a.batch, 65, 256, 256, generator=g).cuda()
    w = (torch.randn(64, 65, 7, 7, generator=g) / 22.6).cuda()
    flop = 2.0 * a.batch * 64 * 128 * 128 * 65 * 49
    res = {"config": f"B={a.batch} 65x256^2 -> 64x128^2, 7x7/2, {a.mode} operands", "flop": flop}
    outs = {}
    f32 = 8 if a.mode == "fp32" else 0  # key 35 mask 8: fp32 gradients, 16: fp32 forward
    for key, name in ((1, "k_conv_lp"), (2 + 3 * f32, "k_conv_stem_lp")):
        old = _lib.call_raw("e2ep_tune", 35, key)
        try:
            with precision.use(a.mode), torch.no_grad():
                for _ in range(5):
                    y = conv.conv2d(x, w, None, (2, 2), (3, 3, 3, 3), (1, 1), 0)
                torch.cuda.synchronize()
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record()
                for _ in range(a.iters):
                    y = conv.conv2d(x, w, None, (2, 2), (3, 3, 3, 3), (1, 1), 0)
                e1.record()
                torch.cuda.synchronize()
            us = e0.elapsed_time(e1) * 1e3 / a.iters
            outs[name] = y
            res[name] = {"us": round(us, 1), "TFLOPs": round(flop / us / 1e6, 1)}
        finally:
            _lib.call_raw("e2ep_tune", 35, old)
    dims = (a.batch, 65, 256, 256, 64, 7, 7, 128, 128, 2, 2, 3, 3, 1, 1)
    wt = conv.tap_major(w)
    gy = torch.randn(a.batch, 64, 128, 128, generator=g).cuda()
    dx = torch.empty(a.batch, 64, 256, 256, device="cuda")
    for key, name in ((1, "dgrad_k_conv_lp"), (4 + f32, "dgrad_k_conv_stem_dgrad_lp")):
        old = _lib.call_raw("e2ep_tune", 35, key)
        try:
            with precision.use(a.mode), torch.no_grad():
                for _ in range(5):
                    conv.conv_dgrad(gy, wt, dims, 64, dx, w_layout=1)
                torch.cuda.synchronize()
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record()
                for _ in range(a.iters):
                    conv.conv_dgrad(gy, wt, dims, 64, dx, w_layout=1)
                e1.record()
                torch.cuda.synchronize()
            us = e0.elapsed_time(e1) * 1e3 / a.iters
            outs[name] = dx.clone()
            res[name] = {"us": round(us, 1), "TFLOPs": round(flop * 64 / 65 / us / 1e6, 1)}
        finally:
            _lib.call_raw("e2ep_tune", 35, old)
    dd = (outs["dgrad_k_conv_stem_dgrad_lp"] - outs["dgrad_k_conv_lp"]).double()
    res["dgrad_rel_l2_direct_vs_gemm"] = (dd.norm() / outs["dgrad_k_conv_lp"].double().norm()).item()
    res["dgrad_speedup"] = round(res["dgrad_k_conv_lp"]["us"] / res["dgrad_k_conv_stem_dgrad_lp"]["us"], 2)
    if a.mode != "fp16":  # the weight gradient (bf16 operands in C3, fp32 in C2)
        dw = torch.empty(64, 65, 7, 7, device="cuda")
        for key, name in ((1, "wgrad_k_wgrad_lp"), (8 + f32, "wgrad_k_conv_stem_wgrad_lp")):
            old = _lib.call_raw("e2ep_tune", 35, key)
            try:
                with precision.use(a.mode), torch.no_grad():
                    for _ in range(5):
                        conv.conv_wgrad(gy, x, dims, dw)
                    torch.cuda.synchronize()
                    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                    e0.record()
                    for _ in range(a.iters):
                        conv.conv_wgrad(gy, x, dims, dw)
                    e1.record()
                    torch.cuda.synchronize()
                us = e0.elapsed_time(e1) * 1e3 / a.iters
                outs[name] = dw.clone()
                res[name] = {"us": round(us, 1), "TFLOPs": round(flop / us / 1e6, 1)}
            finally:
                _lib.call_raw("e2ep_tune", 35, old)
        dd = (outs["wgrad_k_conv_stem_wgrad_lp"] - outs["wgrad_k_wgrad_lp"]).double()
        res["wgrad_rel_l2_direct_vs_gemm"] = (dd.norm() / outs["wgrad_k_wgrad_lp"].double().norm()).item()
        res["wgrad_speedup"] = round(res["wgrad_k_wgrad_lp"]["us"] / res["wgrad_k_conv_stem_wgrad_lp"]["us"], 2)
    d = (outs["k_conv_stem_lp"] - outs["k_conv_lp"]).double()
    res["rel_l2_direct_vs_gemm"] = (d.norm() / outs["k_conv_lp"].double().norm()).item()
    res["speedup"] = round(res["k_conv_lp"]["us"] / res["k_conv_stem_lp"]["us"], 2)
    print(json.dumps(res))


if __name__ == "__main__":
    main()
