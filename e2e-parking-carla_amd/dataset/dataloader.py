"""ParkingDataModule — drop-in for the reference's dataset/dataloader.py.

Same class, constructor and hooks as the reference (dataset/dataloader.py:12-49): setup()
builds CarlaDataset(root, 1, cfg) / CarlaDataset(root, 0, cfg) and torch DataLoaders with
batch_size = cfg.batch_size, shuffle (train only), 8 workers, pinned memory, seed_worker,
drop_last.  It subclasses pytorch_lightning.LightningDataModule when PL is importable (it is
not in this image; the hooks are the same either way).

MI355X path (optional config keys, absent from the reference's YAML):
  frame_cache: <dir>   build (once) / reuse a uint8 frame cache under <dir>/{train,val} and
                       serve batches with GpuFrameLoader — decode on the GPU, batches already
                       in HBM (dataset/frame_cache.py);
  frame_cache_resident: true   keep the whole cache in HBM;
  num_workers: N       DataLoader / cache-build workers (default 8, the reference's value).
"""
import os
import random

import numpy as np
import torch
from torch.utils.data import DataLoader

from dataset.carla_dataset import CarlaDataset

try:  # the reference's base class, when present
    import pytorch_lightning as _pl
    _Base = _pl.LightningDataModule
except ImportError:  # pragma: no cover - PL is absent from this image
    _Base = object


def seed_worker(worker_id):
    """Seed numpy / random in each worker from torch's per-worker seed
    (dataset/dataloader.py:12-15)."""
    worker_seed = torch.initial_seed() % 2 ** 32
    np.random.seed(worker_seed)
    random.seed(worker_seed)


class ParkingDataModule(_Base):
    def __init__(self, cfg):
        super().__init__()
        self.cfg = cfg
        self.data_dir = self.cfg.data_dir
        self.train_loader = None
        self.val_loader = None

    def _loader(self, dataset, shuffle):
        return DataLoader(dataset=dataset, batch_size=self.cfg.batch_size, shuffle=shuffle,
                          num_workers=getattr(self.cfg, "num_workers", None) or 8,
                          pin_memory=True, worker_init_fn=seed_worker, drop_last=True)

    def _cached_loader(self, dataset, split, shuffle):
        """Under DDP every rank runs setup(): rank 0 alone (re)builds the cache when it is
        missing or was built from another dataset / config (frame_cache.cache_matches), the
        others wait for it by polling the file system (frame_cache.wait_for_cache: a build
        can take longer than a collective's watchdog timeout, so no barrier on the process
        group) and then open it read-only — and every rank refuses a cache that does not match
        rather than train on stale frames."""
        from dataset.frame_cache import (FrameCache, GpuFrameLoader, build_frame_cache,
                                         cache_matches, wait_for_cache)
        path = os.path.join(self.cfg.frame_cache, split)
        dist = torch.distributed
        ddp = dist.is_available() and dist.is_initialized()
        rank = dist.get_rank() if ddp else 0
        world = dist.get_world_size() if ddp else 1
        if rank == 0 and not cache_matches(path, dataset):
            build_frame_cache(dataset, path, workers=getattr(self.cfg, "num_workers", None) or 8)
        elif rank != 0:
            wait_for_cache(path, dataset)
        if not cache_matches(path, dataset):
            raise RuntimeError(f"frame cache {path} does not match the {split} dataset "
                               "(built from another dataset or config)")
        cache = FrameCache(path)
        return GpuFrameLoader(cache, self.cfg.batch_size, shuffle=shuffle, drop_last=True,
                              seed=42, resident=bool(getattr(self.cfg, "frame_cache_resident",
                                                             False)),
                              rank=rank, world=world)

    def setup(self, stage=None):
        train_set = CarlaDataset(self.data_dir, 1, self.cfg)
        val_set = CarlaDataset(self.data_dir, 0, self.cfg)
        if getattr(self.cfg, "frame_cache", None):
            self.train_loader = self._cached_loader(train_set, "train", True)
            self.val_loader = self._cached_loader(val_set, "val", False)
        else:
            self.train_loader = self._loader(train_set, True)
            self.val_loader = self._loader(val_set, False)

    def train_dataloader(self):
        return self.train_loader

    def val_dataloader(self):
        return self.val_loader
