"""The reference data path (dataset/carla_dataset.py, dataset/dataloader.py) and the MI355X
frame cache, on the CPU.

Parity anchor: tests/golden/dataset_golden.json, made by running the reference's own
CarlaDataset over the same deterministic mini dataset (tests/golden/make_dataset_golden.py;
carla / torchvision stubs documented there).  Every sample tensor must be bit-identical
(SHA-256) to the reference's; the small label tensors are also compared value by value."""
import hashlib
import json
import os

import numpy as np
import pytest
import torch

import carla_fixture

GOLDEN = os.path.join(os.path.dirname(__file__), "golden", "dataset_golden.json")


def _sha(t):
    return hashlib.sha256(np.ascontiguousarray(t.numpy()).tobytes()).hexdigest()


@pytest.fixture(scope="module")
def golden():
    with open(GOLDEN) as f:
        return json.load(f)


@pytest.fixture(scope="module")
def root(tmp_path_factory, golden):
    d = str(tmp_path_factory.mktemp("carla"))
    carla_fixture.make_dataset(d, frames=golden["frames"])
    return d


@pytest.fixture(scope="module")
def cfg(root):
    return carla_fixture.config(root, batch_size=4, num_workers=2)


@pytest.mark.parametrize("split,is_train", [("train", 1), ("val", 0)])
def test_samples_bit_identical_to_reference(root, cfg, golden, split, is_train):
    from dataset.carla_dataset import CarlaDataset
    ds = CarlaDataset(root, is_train, cfg)
    g = golden["splits"][split]
    assert len(ds) == g["len"]
    seen = set()
    for i in range(len(ds)):
        key = os.path.relpath(str(ds.topdown[i]), root)
        ref = g["samples"][key]
        seen.add(key)
        s = ds[i]
        assert sorted(s) == sorted(ref)
        for k, v in s.items():
            assert str(v.dtype).replace("torch.", "") == ref[k]["dtype"], k
            assert list(v.shape) == ref[k]["shape"], k
            if "values" in ref[k]:
                assert v.reshape(-1).tolist() == ref[k]["values"], k
            assert _sha(v) == ref[k]["sha256"], (key, k)
    assert seen == set(g["samples"])
    assert ds.intrinsic.tolist() == g["intrinsics"]
    assert ds.extrinsic.tolist() == g["extrinsics"]


def test_sample_order_is_listdir_order(root, cfg):
    """Index -> sample follows os.listdir of town / route / task, like the reference."""
    from dataset.carla_dataset import CarlaDataset
    ds = CarlaDataset(root, 1, cfg)
    town = os.path.join(root, cfg.training_map)
    tasks = [os.path.join(town, r, t) for r in os.listdir(town) for t in os.listdir(os.path.join(town, r))]
    per = len(ds) // len(tasks)
    for j, t in enumerate(tasks):
        for k in range(per):
            assert str(ds.front[j * per + k]) == t + f"/rgb_front/{10 + k:04d}.png"


def test_token_helpers_match_reference(golden):
    from dataset.carla_dataset import detokenize, tokenize
    for args, want in golden["helpers"]["tokenize"]:
        assert tokenize(*args, token_nums=204) == want, args
    for toks, want in golden["helpers"]["detokenize"]:
        got = detokenize(toks, token_nums=204)
        assert got == want and all(type(a) is type(b) for a, b in zip(got, want)), toks


def test_process_image_accepts_carla_bgra_frames(root, cfg):
    """The agent feeds carla.Image sensor frames (BGRA raw_data) to ProcessImage
    (dataset/carla_dataset.py:505-509): same result as the decoded PNG."""
    from PIL import Image
    from dataset.carla_dataset import CarlaDataset, ProcessImage
    ds = CarlaDataset(root, 1, cfg)
    rgb = np.asarray(Image.open(str(ds.front[0])).convert("RGB"))
    bgra = np.concatenate([rgb[:, :, ::-1], np.full(rgb.shape[:2] + (1,), 255, np.uint8)], -1)
    frame = type("F", (), {"raw_data": bgra.tobytes(), "height": rgb.shape[0], "width": rgb.shape[1]})
    p = ProcessImage(256)
    a, ca = p(frame)
    b, cb = p(str(ds.front[0]))
    assert torch.equal(a, b) and np.array_equal(ca, cb)


def test_depth_from_rgb_is_reference_formula():
    from dataset.carla_dataset import depth_from_rgb
    rgb = np.random.default_rng(0).integers(0, 256, (5, 7, 3), dtype=np.uint8)
    want = np.dot(rgb.astype(np.float32), [1.0, 256.0, 65536.0])
    want /= (256 * 256 * 256 - 1)
    want = 1000 * want
    got = depth_from_rgb(rgb)
    assert got.dtype == np.float64 and np.array_equal(got, want)
    top = depth_from_rgb(np.full((1, 1, 3), 255, np.uint8))
    assert top[0, 0] == 1000.0


def test_datamodule_reference_loaders(root, cfg):
    from dataset.dataloader import ParkingDataModule
    dm = ParkingDataModule(cfg)
    dm.setup("fit")
    tl, vl = dm.train_dataloader(), dm.val_dataloader()
    assert tl.batch_size == 4 and tl.drop_last and vl.drop_last
    assert len(tl) == 2 and len(vl) == 0          # 8 train samples, 2 val samples < batch
    batch = next(iter(tl))
    assert batch["image"].shape == (4, 4, 3, 256, 256) and batch["image"].dtype == torch.float32
    assert batch["depth"].shape == (4, 4, 256, 256) and batch["depth"].dtype == torch.float64
    assert batch["segmentation"].shape == (4, 1, 200, 200)
    assert batch["extrinsics"].shape == (4, 4, 4, 4) and batch["intrinsics"].shape == (4, 4, 3, 3)
    assert batch["gt_control"].shape == (4, 15) and batch["ego_motion"].shape == (4, 1, 3)


def test_frame_cache_holds_the_reference_inputs(root, cfg, tmp_path):
    from dataset.carla_dataset import (CAMERAS, CarlaDataset, depth_from_rgb, load_depth_rgb,
                                       load_rgb, normalise_image)
    from dataset.frame_cache import FrameCache, build_frame_cache
    ds = CarlaDataset(root, 1, cfg)
    cache = build_frame_cache(ds, str(tmp_path / "fc"), workers=2, chunk=3)
    again = FrameCache(str(tmp_path / "fc"))
    assert len(cache) == len(again) == len(ds)
    for i in range(len(ds)):
        s = ds[i]
        r = again[i]
        for k, cam in enumerate(CAMERAS):
            rgb = r["rgb"][k].numpy()
            assert np.array_equal(rgb, load_rgb(getattr(ds, cam)[i], 256))
            # the cached bytes reproduce the reference tensors exactly
            assert torch.equal(normalise_image(rgb), s["image"][k])
            drgb = r["depth_rgb"][k].numpy()
            assert np.array_equal(drgb, load_depth_rgb(getattr(ds, cam + "_depth")[i], 256))
            assert torch.equal(torch.from_numpy(depth_from_rgb(drgb)), s["depth"][k])
        assert torch.equal(r["bev"].long(), s["segmentation"][0])
        for k in ("target_point", "ego_motion", "gt_control", "gt_acc", "gt_steer", "gt_reverse"):
            assert torch.equal(r[k], s[k]), k
    assert torch.equal(again.intrinsics, ds.intrinsic) and torch.equal(again.extrinsics, ds.extrinsic)
    g = again.gather(np.array([3, 1]))
    assert np.array_equal(g["rgb"][0], again.arrays["rgb"][3])


def test_frame_cache_reuse_is_validated(root, cfg, tmp_path):
    """A cache directory is reused only when it is complete (meta.json, written last and
    atomically) and was built from the same dataset (fingerprint of count, crop, rig, frame paths
    and label / measurement rows); another split, changed labels, moved frames or changed
    accelerations do not match, and a rebuild invalidates first."""
    from dataset.carla_dataset import CarlaDataset
    from dataset.frame_cache import build_frame_cache, cache_matches
    path = str(tmp_path / "fc")
    ds = CarlaDataset(root, 1, cfg)
    assert not cache_matches(path, ds)
    build_frame_cache(ds, path, chunk=4)
    assert cache_matches(path, ds)
    assert not any(f.startswith("meta.json.tmp") for f in os.listdir(path))
    assert not cache_matches(path, CarlaDataset(root, 0, cfg))
    changed = CarlaDataset(root, 1, cfg)
    changed.target_point = changed.target_point + 1.0
    assert not cache_matches(path, changed)
    # same labels, other frames (another image set / root) or other ego accelerations
    moved = CarlaDataset(root, 1, cfg)
    moved.front = np.array([f.replace("rgb_front", "rgb_front_other") for f in moved.front])
    assert not cache_matches(path, moved)
    acc = CarlaDataset(root, 1, cfg)
    acc.acc_y = acc.acc_y + 0.5
    assert not cache_matches(path, acc)


def _cache_rank(rank, world, port, root, cfg, path, out):
    """One rank of the frame-cache setup under a process group whose collective timeout (2 s)
    is shorter than rank 0's cache build (5 s)."""
    import datetime
    import time
    import torch.distributed as dist
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world,
                            timeout=datetime.timedelta(seconds=2))
    from dataset import frame_cache
    from dataset.dataloader import ParkingDataModule
    from dataset.carla_dataset import CarlaDataset
    real_build = frame_cache.build_frame_cache

    def slow_build(*a, **k):
        time.sleep(5.0)
        return real_build(*a, **k)

    frame_cache.build_frame_cache = slow_build
    frame_cache.GpuFrameLoader = lambda cache, *a, **k: ("loader", len(cache), k["rank"], k["world"])
    cfg.frame_cache = path
    got = ParkingDataModule(cfg)._cached_loader(CarlaDataset(root, 1, cfg), "train", True)
    dist.barrier()  # the group is still healthy after the long build
    out[rank] = got
    dist.destroy_process_group()


def test_ddp_cache_build_outlasts_collective_timeout(root, cfg, tmp_path):
    """under DDP rank 0 builds the frame cache while the other ranks wait.  They
    wait by polling the file system (frame_cache.wait_for_cache), not in a collective, so a
    build longer than the process group's timeout does not abort them."""
    import copy
    import socket
    import torch.multiprocessing as mp
    with socket.socket() as so:
        so.bind(("127.0.0.1", 0))
        port = so.getsockname()[1]
    with mp.Manager() as man:
        out = man.dict()
        mp.spawn(_cache_rank, args=(2, port, root, copy.copy(cfg), str(tmp_path / "fc"), out),
                 nprocs=2, join=True)
        res = dict(out)
    assert res[0][0] == res[1][0] == "loader" and res[0][1] == res[1][1] > 0
    assert (res[0][2], res[1][2]) == (0, 1) and res[0][3] == res[1][3] == 2


def test_frame_cache_empty_split(tmp_path, cfg):
    from dataset.carla_dataset import CarlaDataset
    from dataset.frame_cache import FrameCache, build_frame_cache
    d = tmp_path / "empty"
    carla_fixture.make_dataset(str(d), frames=14, layout={carla_fixture.TRAIN_TOWN: {"r": ["t"]}})
    ds = CarlaDataset(str(d), 1, cfg)          # 14 frames: no frame in [10, 10)
    assert len(ds) == 0
    build_frame_cache(ds, str(tmp_path / "fc"))
    assert len(FrameCache(str(tmp_path / "fc"))) == 0


@pytest.mark.parametrize("n,B,world,drop", [(10, 4, 1, True), (10, 4, 1, False), (11, 2, 2, True),
                                            (7, 3, 3, False)])
def test_epoch_indices_cover_and_shard(n, B, world, drop):
    from dataset.frame_cache import epoch_indices
    per_rank = [epoch_indices(n, B, True, drop, 42, 0, r, world) for r in range(world)]
    flat = [int(i) for r in per_rank for b in r for i in b]
    assert all(len(b) == B for r in per_rank for b in r) or not drop
    if not drop:
        assert set(flat) == set(range(n))
    m = -(-n // world)
    assert all(len(r) == (m // B if drop else -(-m // B)) for r in per_rank)
    a = epoch_indices(n, B, True, drop, 42, 1)
    b = epoch_indices(n, B, True, drop, 42, 1)
    assert all(torch.equal(x, y) for x, y in zip(a, b))
