"""The MI355X frame cache: the reference data path with its per-step CPU work moved off it.

The reference re-decodes 8 PNGs and a BEV image per sample every epoch in 8 CPU worker
processes (dataset/carla_dataset.py:379-423, dataset/dataloader.py:30-43), then ships fp32
images and float64 depth over PCIe.  Every step of that is a pure function of the files on
disk, so here it is split in two:

  build_frame_cache(dataset, dir)   once: PNG decode + nearest resize + centre crop + slot
                                    drawing on the CPU (the reference's own helpers), stored as
                                    uint8 .npy arrays — 1.61 MB per sample at the C3 config:
        rgb        (N, 4, crop, crop, 3) u8   cropped camera frames
        depth_rgb  (N, 4, crop, crop, 3) u8   cropped CARLA depth encodings
        bev        (N, 200, 200)         u8   BEV classes {0, 1, 2} (ProcessSemantic output)
        target_point (N, 3) f32, ego_motion (N, 1, 3) f32, gt_control (N, T) i64,
        gt_acc / gt_steer (N, F) f32, gt_reverse (N, F) i64
  GpuFrameLoader(cache, ...)        per step: batch index -> uint8 rows -> HBM -> the HIP
                                    decode kernels (csrc/decode.hip) produce the reference
                                    batch (image fp32 normalised, depth fp64 metres,
                                    segmentation i64, ...) bit-identical to collating
                                    CarlaDataset samples.

`resident=True` uploads the whole cache to HBM once (288 GB holds ~170k samples) and each
batch is a gather+decode kernel reading the resident pixels directly; otherwise a host thread
gathers rows out of the memory-mapped arrays into pinned slots and a side stream copies them
(uint8: 4x fewer PCIe bytes than the reference's fp32 / fp64 tensors).
"""
import json
import os
import queue
import threading

import numpy as np
import torch

from dataset.carla_dataset import CAMERAS, load_depth_rgb, load_rgb

VERSION = 1
BEV = 200
PIXEL_FIELDS = ("rgb", "depth_rgb")
LABEL_FIELDS = ("target_point", "ego_motion", "gt_control", "gt_acc", "gt_steer", "gt_reverse")


def _tdtype(a):
    return torch.from_numpy(np.empty(0, dtype=a.dtype)).dtype


def _layout(n, crop, tokens, future):
    return {
        "rgb": (np.uint8, (n, 4, crop, crop, 3)),
        "depth_rgb": (np.uint8, (n, 4, crop, crop, 3)),
        "bev": (np.uint8, (n, BEV, BEV)),
        "target_point": (np.float32, (n, 3)),
        "ego_motion": (np.float32, (n, 1, 3)),
        "gt_control": (np.int64, (n, tokens)),
        "gt_acc": (np.float32, (n, future)),
        "gt_steer": (np.float32, (n, future)),
        "gt_reverse": (np.int64, (n, future)),
    }


def _fill(dataset, out_dir, lo, hi):
    """Decode samples [lo, hi) into the cache arrays (opened read-write in this process)."""
    arr = {f: np.load(os.path.join(out_dir, f + ".npy"), mmap_mode="r+")
           for f in ("rgb", "depth_rgb", "bev")}
    crop = dataset.image_crop
    for i in range(lo, hi):
        for k, cam in enumerate(CAMERAS):
            arr["rgb"][i, k] = load_rgb(getattr(dataset, cam)[i], crop)
            arr["depth_rgb"][i, k] = load_depth_rgb(getattr(dataset, cam + "_depth")[i], crop)
        seg = dataset.semantic_process(dataset.topdown[i], scale=0.5, crop=BEV,
                                       target_slot=dataset.target_point[i])
        arr["bev"][i] = seg.astype(np.uint8)
    for a in arr.values():
        a.flush()


_BUILD = None  # the dataset being cached, inherited by forked workers


def _fill_worker(args):
    _fill(_BUILD, *args)


def build_frame_cache(dataset, out_dir, workers=0, chunk=32):
    """Decode every sample of a CarlaDataset once into `out_dir` and return the FrameCache.
    workers > 1 forks that many decoder processes (build before touching the GPU)."""
    global _BUILD
    os.makedirs(out_dir, exist_ok=True)
    meta_path = os.path.join(out_dir, "meta.json")
    if os.path.exists(meta_path):  # a cache being rebuilt is not a cache until meta.json is back
        os.remove(meta_path)
    n = len(dataset)
    crop = dataset.image_crop
    tokens = dataset.control.shape[1] if n else 3 * dataset.cfg.future_frame_nums + 3
    future = dataset.cfg.future_frame_nums
    layout = _layout(n, crop, tokens, future)
    if n == 0:  # nothing to map: write empty arrays
        for f, (dt, shape) in layout.items():
            np.save(os.path.join(out_dir, f + ".npy"), np.empty(shape, dtype=dt))
        arrays = {}
    else:
        arrays = {f: np.lib.format.open_memmap(os.path.join(out_dir, f + ".npy"), mode="w+",
                                               dtype=dt, shape=shape)
                  for f, (dt, shape) in layout.items()}
    if n:
        arrays["target_point"][:] = dataset.target_point
        arrays["ego_motion"][:] = np.stack([dataset.velocity, dataset.acc_x, dataset.acc_y],
                                           axis=1)[:, None, :]
        arrays["gt_control"][:] = dataset.control
        arrays["gt_acc"][:] = dataset.throttle_brake
        arrays["gt_steer"][:] = dataset.steer
        arrays["gt_reverse"][:] = dataset.reverse
    for a in arrays.values():
        a.flush()
    del arrays
    spans = [(lo, min(lo + chunk, n)) for lo in range(0, n, chunk)]
    if workers > 1 and len(spans) > 1:
        import multiprocessing as mp
        _BUILD = dataset
        try:
            with mp.get_context("fork").Pool(workers) as pool:
                pool.map(_fill_worker, [(out_dir, lo, hi) for lo, hi in spans])
        finally:
            _BUILD = None
    else:
        for lo, hi in spans:
            _fill(dataset, out_dir, lo, hi)
    meta = {"version": VERSION, "samples": n, "image_crop": crop, "bev": BEV,
            "intrinsics": dataset.intrinsic.tolist(), "extrinsics": dataset.extrinsic.tolist(),
            "fingerprint": dataset_fingerprint(dataset),
            "fields": {f: [np.dtype(dt).str, list(shape)] for f, (dt, shape) in layout.items()}}
    # meta.json last and atomically: its presence means every array above is complete
    tmp = meta_path + f".tmp{os.getpid()}"
    with open(tmp, "w") as f:
        json.dump(meta, f)
    os.replace(tmp, meta_path)
    return FrameCache(out_dir)


# every per-sample field a cache is built from, without decoding any frame: the frame file
# paths (camera, depth and BEV images) and every label / measurement row
_FINGERPRINT_FIELDS = ("intrinsic", "extrinsic", "front", "left", "right", "rear", "front_depth",
                       "left_depth", "right_depth", "rear_depth", "topdown", "target_point",
                       "control", "velocity", "acc_x", "acc_y", "throttle_brake", "steer",
                       "reverse")


def dataset_fingerprint(dataset):
    """SHA-256 over what identifies a CarlaDataset's samples without decoding any frame: the
    sample count, crop, rig, the frame file paths of every sample (so a cache built from
    another image set or root does not match) and the per-sample label / measurement rows
    (acc_x / acc_y included: they feed ego_motion).  A cache whose fingerprint differs belongs
    to another dataset or config."""
    import hashlib
    h = hashlib.sha256()
    h.update(repr((len(dataset), int(dataset.image_crop))).encode())
    for name in _FINGERPRINT_FIELDS:
        a = np.ascontiguousarray(np.asarray(getattr(dataset, name)))
        h.update(name.encode() + a.dtype.str.encode() + repr(a.shape).encode() + a.tobytes())
    return h.hexdigest()


def wait_for_cache(path, dataset, timeout_s=None, poll_s=2.0):
    """Block until `path` holds a complete cache built from `dataset` (cache_matches), polling
    the file system — the non-building ranks of a data-parallel job wait here while rank 0
    builds it, instead of in a collective whose watchdog would time out a long build.  Raises
    TimeoutError after `timeout_s` (default: E2EP_CACHE_WAIT_S or 24 h)."""
    import time
    if timeout_s is None:
        timeout_s = float(os.environ.get("E2EP_CACHE_WAIT_S", 24 * 3600))
    t_end = time.monotonic() + timeout_s
    while not cache_matches(path, dataset):
        if time.monotonic() > t_end:
            raise TimeoutError(f"frame cache {path}: no matching cache after {timeout_s:.0f} s")
        time.sleep(poll_s)


def cache_matches(path, dataset):
    """True when `path` holds a complete cache (meta.json present) built from `dataset`."""
    meta_path = os.path.join(path, "meta.json")
    if not os.path.exists(meta_path):
        return False
    with open(meta_path) as f:
        meta = json.load(f)
    return (meta.get("version") == VERSION and meta.get("samples") == len(dataset)
            and meta.get("image_crop") == dataset.image_crop
            and meta.get("fingerprint") == dataset_fingerprint(dataset))


class FrameCache(torch.utils.data.Dataset):
    """A built cache, memory-mapped.  Indexing returns one sample's raw uint8 / label rows
    (for any torch DataLoader); GpuFrameLoader turns batches into reference tensors."""

    def __init__(self, path):
        with open(os.path.join(path, "meta.json")) as f:
            self.meta = json.load(f)
        if self.meta.get("version") != VERSION:
            raise ValueError(f"frame cache {path}: version {self.meta.get('version')} != {VERSION}")
        self.path = path
        mode = "r" if self.meta["samples"] else None
        self.arrays = {name: np.load(os.path.join(path, name + ".npy"), mmap_mode=mode)
                       for name in self.meta["fields"]}
        for name, (dt, shape) in self.meta["fields"].items():
            a = self.arrays[name]
            if a.dtype.str != dt or list(a.shape) != shape:
                raise ValueError(f"frame cache {path}: {name} is {a.dtype}{a.shape}, "
                                 f"meta says {dt}{shape}")
        self.crop = self.meta["image_crop"]
        self.intrinsics = torch.tensor(self.meta["intrinsics"], dtype=torch.float32)
        self.extrinsics = torch.tensor(self.meta["extrinsics"], dtype=torch.float32)

    def __len__(self):
        return self.meta["samples"]

    def __getitem__(self, i):
        return {k: torch.from_numpy(np.array(a[i])) for k, a in self.arrays.items()}

    def gather(self, idx, out=None):
        """Rows `idx` of every field as numpy arrays (into `out` when given)."""
        out = out if out is not None else {}
        for k, a in self.arrays.items():
            dst = out.get(k)
            if dst is None:
                out[k] = a[idx]
            else:
                np.take(a, idx, axis=0, out=dst[:len(idx)])
        return out

    @property
    def nbytes(self):
        return sum(a.nbytes for a in self.arrays.values())


def epoch_indices(n, batch_size, shuffle, drop_last, seed, epoch, rank=0, world=1):
    """This rank's sample order for one epoch: a seeded permutation (torch.randperm, as
    DataLoader's RandomSampler), padded to a multiple of `world` and strided over ranks like
    torch's DistributedSampler; then cut into batches (the last partial one dropped when
    drop_last, as the reference's loaders do, dataset/dataloader.py:36,43)."""
    if shuffle:
        order = torch.randperm(n, generator=torch.Generator().manual_seed(seed + epoch))
    else:
        order = torch.arange(n)
    if world > 1:
        pad = (-n) % world
        if pad:
            order = torch.cat([order, order[:pad]])
        order = order[rank::world]
    m = len(order)
    stop = m - m % batch_size if drop_last else m
    return [order[i:i + batch_size] for i in range(0, stop, batch_size)]


class GpuFrameLoader:
    """Iterate reference-schema batches of a FrameCache, already on the HIP device.

    Each batch dict has the keys and dtypes the reference's DataLoader collates
    (dataset/carla_dataset.py:379-423): image (B,4,3,C,C) f32, depth (B,4,C,C) f64,
    segmentation (B,1,200,200) i64, extrinsics (B,4,4,4) / intrinsics (B,4,3,3) f32,
    target_point (B,3), ego_motion (B,1,3), gt_control (B,T), gt_acc / gt_steer (B,F),
    gt_reverse (B,F).  The camera rig (intrinsics / extrinsics) is constant per cache and
    stays on the host by default (rig_on_host), where the model's LSS plan cache keys on it
    (model/bev_model.py plan()); every other tensor is on the device."""

    def __init__(self, cache, batch_size, shuffle=True, drop_last=True, seed=0, device=None,
                 resident=False, rank=0, world=1, prefetch=2, rig_on_host=True):
        if not torch.cuda.is_available():
            from e2ep_amd import _lib
            raise _lib.E2EPError("GpuFrameLoader needs a HIP device")
        self.cache = cache
        self.batch_size = int(batch_size)
        self.shuffle, self.drop_last, self.seed = shuffle, drop_last, seed
        self.device = torch.device(device if device is not None else "cuda")
        self.resident = resident
        self.rank, self.world = rank, world
        self.prefetch = max(1, int(prefetch))
        self.rig_on_host = rig_on_host
        self.epoch = 0
        self._dev = None
        self._rig = {}

    def set_epoch(self, epoch):
        self.epoch = int(epoch)

    def batches(self):
        return epoch_indices(len(self.cache), self.batch_size, self.shuffle, self.drop_last,
                             self.seed, self.epoch, self.rank, self.world)

    def __len__(self):
        return len(self.batches())

    def _rig_for(self, B):
        if B not in self._rig:
            where = "cpu" if self.rig_on_host else self.device
            ex = self.cache.extrinsics.to(where)
            ki = self.cache.intrinsics.to(where)
            self._rig[B] = (ex.unsqueeze(0).expand(B, -1, -1, -1).contiguous(),
                            ki.unsqueeze(0).expand(B, -1, -1, -1).contiguous())
        return self._rig[B]

    def upload(self, slab_mb=256):
        """Make the whole cache resident in HBM (slab by slab, so host memory stays flat)."""
        if self._dev is None:
            dev = {}
            for k, a in self.cache.arrays.items():
                t = torch.empty(a.shape, dtype=_tdtype(a), device=self.device)
                rows = max(1, (slab_mb << 20) // max(1, a[0].nbytes if len(a) else 1))
                for lo in range(0, len(a), rows):
                    t[lo:lo + rows].copy_(torch.from_numpy(np.ascontiguousarray(a[lo:lo + rows])))
                dev[k] = t
            self._dev = dev
        return self._dev

    def _assemble(self, rgb, depth_rgb, bev, labels, B, src=None, src_frames=None):
        from e2ep_amd import decode
        C = self.cache.crop
        image, depth = decode.decode_frames(rgb.view(-1, C, C, 3), depth_rgb.view(-1, C, C, 3),
                                            src_frame=src_frames)
        seg = decode.widen_rows(bev, src_row=src)
        ex, ki = self._rig_for(B)
        batch = {"image": image.view(B, 4, 3, C, C), "depth": depth.view(B, 4, C, C),
                 "extrinsics": ex, "intrinsics": ki,
                 "segmentation": seg.view(B, 1, BEV, BEV)}
        batch.update(labels)
        return batch

    def _iter_resident(self):
        dev = self.upload()
        for idx in self.batches():
            B = len(idx)
            frames = (idx[:, None] * 4 + torch.arange(4)).reshape(-1)
            didx = idx.to(self.device, non_blocking=True)
            labels = {k: dev[k].index_select(0, didx) for k in LABEL_FIELDS}
            yield self._assemble(dev["rgb"], dev["depth_rgb"], dev["bev"], labels, B,
                                 src=idx, src_frames=frames)

    def _iter_streamed(self):
        batches = self.batches()
        if not batches:
            return
        width = max(len(b) for b in batches)
        slots = []
        for _ in range(self.prefetch + 1):
            slots.append({k: torch.empty((width,) + a.shape[1:],
                                         dtype=_tdtype(a)).pin_memory()
                          for k, a in self.cache.arrays.items()})
        # The producer thread only gathers rows on the host (numpy), never calls HIP: a slot
        # comes back to it through `free` after the main thread has seen the slot's H2D copy
        # complete, so no thread but the caller's touches the device (a HIP call from a helper
        # thread would break a graph capture running on the main thread).
        free, ready = queue.Queue(), queue.Queue()
        for s in range(len(slots)):
            free.put(s)
        stop = threading.Event()

        def producer():
            try:
                for idx in batches:
                    s = free.get()
                    if stop.is_set():
                        return
                    self.cache.gather(idx.numpy(),
                                      out={k: v.numpy() for k, v in slots[s].items()})
                    ready.put((s, len(idx)))
            except BaseException as e:  # surface in the consumer
                ready.put(e)
            ready.put(None)

        th = threading.Thread(target=producer, daemon=True)
        th.start()
        copy = torch.cuda.Stream(self.device)
        main = torch.cuda.current_stream(self.device)
        inflight = []  # (slot, event of its H2D copy), oldest first
        try:
            while True:
                item = ready.get()
                if item is None:
                    break
                if isinstance(item, BaseException):
                    raise item
                s, B = item
                with torch.cuda.stream(copy):
                    host = slots[s]
                    d = {k: v[:B].to(self.device, non_blocking=True) for k, v in host.items()}
                    ev = torch.cuda.Event()
                    ev.record(copy)
                main.wait_event(ev)
                for t in d.values():
                    t.record_stream(main)
                inflight.append((s, ev))
                # hand back the slots whose copies are done (keep at most one in flight)
                while len(inflight) > 1 or (inflight and inflight[0][1].query()):
                    s0, e0 = inflight.pop(0)
                    e0.synchronize()
                    free.put(s0)
                labels = {k: d[k] for k in LABEL_FIELDS}
                yield self._assemble(d["rgb"], d["depth_rgb"], d["bev"], labels, B)
        finally:
            stop.set()
            for s in range(len(slots)):
                free.put(s)
            th.join(timeout=10)

    def __iter__(self):
        it = self._iter_resident() if self.resident else self._iter_streamed()
        yield from it
        self.epoch += 1
