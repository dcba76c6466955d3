"""Data-path throughput: the reference loader vs the MI355X frame cache.

Builds a deterministic mini CARLA dataset (tests/carla_fixture.py layout and PNG sizes), then
measures samples/s delivered ON THE DEVICE in the reference batch schema:
  reference   CarlaDataset + DataLoader(batch, 8 workers, pinned, drop_last) as
              dataset/dataloader.py:30-36 configures it, each batch moved to the GPU
              (what PL does before training_step); one epoch incl. worker start-up;
  build       build_frame_cache (one-time PNG decode into uint8 arrays);
  streamed    GpuFrameLoader over the memory-mapped cache (host gather -> pinned -> H2D ->
              HIP decode);
  resident    GpuFrameLoader with the cache resident in HBM (gather+decode kernel);
  kernel      e2ep_decode_frames alone at the batch size, HIP events: algorithmic bytes
              (26 B per camera pixel: 6 read, 12 + 8 written) / time vs 8 TB/s.
Prints one JSON line (and writes it to --out).
"""
import argparse
import json
import os
import sys
import tempfile
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (os.path.join(ROOT, "tests"), os.path.join(ROOT, "e2e-parking-carla_amd"), ROOT):
    sys.path.insert(0, p)

import torch  # noqa: E402

import carla_fixture  # noqa: E402


def to_dev(batch):
    return {k: v.to("cuda", non_blocking=True) for k, v in batch.items()}


def timed_epochs(loader, epochs, move=False):
    n = 0
    t0 = time.perf_counter()
    for _ in range(epochs):
        for b in loader:
            if move:
                b = to_dev(b)
            n += b["image"].shape[0]
    torch.cuda.synchronize()
    return n / (time.perf_counter() - t0), n


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--routes", type=int, default=4)
    ap.add_argument("--tasks", type=int, default=4)
    ap.add_argument("--frames", type=int, default=24)
    ap.add_argument("--batch", type=int, default=8)
    ap.add_argument("--workers", type=int, default=8)
    ap.add_argument("--out", default=None)
    args = ap.parse_args()

    from torch.utils.data import DataLoader
    from dataset.carla_dataset import CarlaDataset
    from dataset.dataloader import seed_worker
    from dataset.frame_cache import GpuFrameLoader, build_frame_cache
    from e2ep_amd import decode

    res = {"metric": "data_samples_per_s", "unit": "samples/s", "batch": args.batch}
    with tempfile.TemporaryDirectory() as root:
        layout = {carla_fixture.TRAIN_TOWN: {f"route_{r}": [f"task_{t}" for t in range(args.tasks)]
                                             for r in range(args.routes)}}
        t0 = time.perf_counter()
        carla_fixture.make_dataset(root, frames=args.frames, layout=layout)
        res["fixture_s"] = round(time.perf_counter() - t0, 2)
        cfg = carla_fixture.config(root, batch_size=args.batch)
        ds = CarlaDataset(root, 1, cfg)
        res["samples"] = len(ds)
        print(f"dataset: {len(ds)} samples", flush=True)

        ref = DataLoader(ds, batch_size=args.batch, shuffle=True, num_workers=args.workers,
                         pin_memory=True, worker_init_fn=seed_worker, drop_last=True)
        timed_epochs(ref, 1, move=True)  # warm the page cache / imports
        v, n = timed_epochs(ref, 2, move=True)
        res["reference"] = {"value": round(v, 1), "workers": args.workers, "samples": n}
        print("reference", res["reference"], flush=True)

        t0 = time.perf_counter()
        cache = build_frame_cache(ds, os.path.join(root, "fc"), workers=args.workers)
        res["build"] = {"seconds": round(time.perf_counter() - t0, 2),
                        "bytes_per_sample": cache.nbytes // max(1, len(cache))}
        print("build", res["build"], flush=True)

        for name, resident in (("streamed", False), ("resident", True)):
            ld = GpuFrameLoader(cache, args.batch, shuffle=True, resident=resident)
            timed_epochs(ld, 1)
            v, n = timed_epochs(ld, 5)
            res[name] = {"value": round(v, 1), "samples": n}
            print(name, res[name], flush=True)

        # the decode kernel alone, batch-sized, resident gather
        ld = GpuFrameLoader(cache, args.batch, resident=True)
        dev = ld.upload()
        C = cache.crop
        frames = (torch.arange(args.batch)[:, None] * 4 + torch.arange(4)).reshape(-1)
        rgb, drgb = dev["rgb"].view(-1, C, C, 3), dev["depth_rgb"].view(-1, C, C, 3)
        for _ in range(5):
            decode.decode_frames(rgb, drgb, src_frame=frames)
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        iters = 200
        e0.record()
        for _ in range(iters):
            decode.decode_frames(rgb, drgb, src_frame=frames)
        e1.record()
        torch.cuda.synchronize()
        ms = e0.elapsed_time(e1) / iters
        nbytes = 26 * frames.numel() * C * C
        res["kernel"] = {"name": "k_decode_frames", "us": round(ms * 1e3, 2),
                         "achieved_GBps": round(nbytes / ms / 1e6, 1), "peak_GBps": 8000.0,
                         "frac": round(nbytes / ms / 1e6 / 8000.0, 3), "bytes": nbytes}
        print("kernel", res["kernel"], flush=True)
    line = json.dumps(res)
    print(line)
    if args.out:
        with open(args.out, "w") as f:
            f.write(line + "\n")


if __name__ == "__main__":
    main()
