"""Generate tests/golden/dataset_golden.json by running the REFERENCE's CarlaDataset
(dataset/carla_dataset.py) over the deterministic mini dataset of tests/carla_fixture.py.

Run in the build container only (needs /root/reference):
    python tests/golden/make_dataset_golden.py

The reference module is imported unmodified.  Its third-party imports are absent from this
image and are provided as follows:
  * carla 0.9.11 (simulator client): Transform / Location / Rotation from
    e2ep_amd.carla_math (float64 restatement of LibCarla's matrix convention) — the CARLA
    matrix arithmetic itself is therefore UNPINNED against a live client;
  * torchvision 0.14.1 (environment.yml:91): transforms.Compose / ToTensor / Normalize
    restated from torchvision's published functional code (ndarray HWC uint8 -> CHW, .float()
    .div(255); sub_(mean[:, None, None]).div_(std[:, None, None]));
  * loguru: a logger whose info() discards;
  * numpy 2 dropped np.string_: aliased to np.bytes_ (the reference's own value type).
The reference pins numpy 1.21, where np.float32 / float promotes to float64 in the slot
drawing (dataset/carla_dataset.py:468-470); this container runs numpy 2 (float32).  The script
asserts the two promotions give the same slot pixel for every sample, so the fixture holds
for both.  Only inputs' descriptions and outputs (SHA-256 of every sample tensor plus the
small label tensors verbatim) are written — no reference source.
"""
import hashlib
import json
import os
import sys
import tempfile
import types

import numpy as np
import torch

REPO = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
REF = "/root/reference"
OUT = os.path.join(REPO, "tests", "golden", "dataset_golden.json")
sys.path.insert(0, os.path.join(REPO, "e2e-parking-carla_amd"))
sys.path.insert(0, os.path.join(REPO, "tests"))

from e2ep_amd import carla_math  # noqa: E402
import carla_fixture  # noqa: E402

LABELS = ("target_point", "ego_motion", "gt_control", "gt_acc", "gt_steer", "gt_reverse")


def install_shims():
    np.string_ = np.bytes_
    carla = types.ModuleType("carla")
    carla.Transform, carla.Location, carla.Rotation = (carla_math.Transform, carla_math.Location,
                                                       carla_math.Rotation)
    carla.Image = type("Image", (), {})
    sys.modules["carla"] = carla

    tv = types.ModuleType("torchvision")
    tvt = types.ModuleType("torchvision.transforms")

    class Compose:
        def __init__(self, fs):
            self.fs = fs

        def __call__(self, x):
            for f in self.fs:
                x = f(x)
            return x

    class ToTensor:
        def __call__(self, pic):
            img = torch.from_numpy(pic.transpose((2, 0, 1))).contiguous()
            return img.to(dtype=torch.get_default_dtype()).div(255)

    class Normalize:
        def __init__(self, mean, std):
            self.mean, self.std = mean, std

        def __call__(self, t):
            t = t.clone()
            mean = torch.as_tensor(self.mean, dtype=t.dtype)
            std = torch.as_tensor(self.std, dtype=t.dtype)
            return t.sub_(mean.view(-1, 1, 1)).div_(std.view(-1, 1, 1))

    tvt.Compose, tvt.ToTensor, tvt.Normalize = Compose, ToTensor, Normalize
    tv.transforms = tvt
    sys.modules.update({"torchvision": tv, "torchvision.transforms": tvt})
    lg = types.ModuleType("loguru")
    lg.logger = types.SimpleNamespace(info=lambda *a, **k: None)
    sys.modules["loguru"] = lg
    prod = os.path.join(REPO, "e2e-parking-carla_amd")
    sys.path[:] = [p for p in sys.path if os.path.abspath(p or ".") != prod]
    for name in list(sys.modules):
        if name.split(".")[0] in ("model", "tool", "loss", "trainer", "dataset"):
            del sys.modules[name]
    sys.path.insert(0, REF)


def sha(t):
    return hashlib.sha256(np.ascontiguousarray(t.numpy()).tobytes()).hexdigest()


def cfg():
    return types.SimpleNamespace(token_nums=204, image_crop=256, hist_frame_nums=10,
                                 future_frame_nums=4, training_map=carla_fixture.TRAIN_TOWN,
                                 validation_map=carla_fixture.VAL_TOWN,
                                 bev_x_bound=[-10.0, 10.0, 0.1], bev_y_bound=[-10.0, 10.0, 0.1])


def main():
    install_shims()
    import dataset.carla_dataset as R   # the reference module

    out = {"generator": "tests/golden/make_dataset_golden.py", "fixture": "tests/carla_fixture.py",
           "frames": 16, "splits": {}, "helpers": {}}
    with tempfile.TemporaryDirectory() as root:
        carla_fixture.make_dataset(root, frames=16)
        c = cfg()
        for split, is_train in (("train", 1), ("val", 0)):
            ds = R.CarlaDataset(root, is_train, c)
            samples = {}
            for i in range(len(ds)):
                tp = ds.target_point[i]
                p32 = np.array([100 - tp[0] / 0.1, 100 + tp[1] / 0.1], dtype=int)
                p64 = np.array([100 - float(tp[0]) / 0.1, 100 + float(tp[1]) / 0.1], dtype=int)
                assert (p32 == p64).all(), "numpy 1.21 / 2.x promotion would differ here"
                s = ds[i]
                key = os.path.relpath(ds.topdown[i].decode(), root)
                e = {k: {"dtype": str(v.dtype).replace("torch.", ""), "shape": list(v.shape),
                         "sha256": sha(v)} for k, v in s.items()}
                for k in LABELS:
                    e[k]["values"] = s[k].reshape(-1).tolist()
                e["image"]["sum"] = float(s["image"].double().sum())
                e["depth"]["sum"] = float(s["depth"].sum())
                e["segmentation"]["counts"] = torch.bincount(s["segmentation"].reshape(-1),
                                                             minlength=3).tolist()
                samples[key] = e
            out["splits"][split] = {"len": len(ds), "samples": samples,
                                    "intrinsics": ds.intrinsic.tolist(),
                                    "extrinsics": ds.extrinsic.tolist()}
    grid = [(t, b, s, r) for t in (0.0, 0.37, 1.0) for b in (0.0, 0.5, 1.0)
            for s in (-1.0, -0.31, 0.0, 0.77, 1.0) for r in (0, 1)]
    out["helpers"]["tokenize"] = [[list(a), R.tokenize(*a, token_nums=204)] for a in grid]
    toks = [[a, b, c] for a in (0, 50, 97, 98, 99, 150, 196) for b in (0, 98, 196) for c in (0, 98, 99)]
    out["helpers"]["detokenize"] = [[t, R.detokenize(t, token_nums=204)] for t in toks]
    with open(OUT, "w") as f:
        json.dump(out, f, indent=0)
    print("wrote", OUT, {k: v["len"] for k, v in out["splits"].items()})


if __name__ == "__main__":
    main()
