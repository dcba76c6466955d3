"""A deterministic, miniature on-disk CARLA parking dataset in the reference's layout
(dataset/carla_dataset.py:272-348, data_generation/data_generator.py:180-300):

  <root>/<town>/<route>/<task>/rgb_{front,left,right,rear}/NNNN.png     400x300 RGB
                               depth_{front,left,right,rear}/NNNN.png   400x300 CARLA depth
                               topdown/encoded_NNNN.png                  200x200 grey BEV
                               measurements/NNNN.json                    ego pose, motion, controls
                               parking_goal/0001.json                    slot pose

Every value is drawn from numpy's PCG64 seeded per file, so the same arguments give the same
bytes on any host.  Used by the dataset parity tests and by tests/golden/make_dataset_golden.py,
which runs the reference's CarlaDataset over it.
"""
import json
import os

import numpy as np
from PIL import Image

CAMS = ("front", "left", "right", "rear")
TRAIN_TOWN, VAL_TOWN = "Town04_Opt", "Town04_Opt_Val"


def _seed(text):
    # stable across processes (str hash is salted): sum of code points weighted by position
    return sum((i + 1) * ord(c) for i, c in enumerate(text)) % (2 ** 31)


def _camera_png(path, g):
    # smooth gradient + blocky noise: realistic enough, cheap to encode
    y, x = np.mgrid[0:300, 0:400]
    base = np.stack([(x * g.integers(1, 4)) % 256, (y * g.integers(1, 4)) % 256,
                     ((x + y) * g.integers(1, 3)) % 256], -1)
    noise = np.kron(g.integers(0, 64, (30, 40, 3)), np.ones((10, 10, 1), dtype=np.int64))
    Image.fromarray(((base + noise) % 256).astype(np.uint8), "RGB").save(path, compress_level=1)


def _depth_png(path, g):
    y, x = np.mgrid[0:300, 0:400]
    metres = 0.3 + 25.0 * (y / 300.0) + g.uniform(0, 3.0, (300, 400))
    metres[:20] = 1000.0                       # sky: far plane
    metres[g.uniform(size=(300, 400)) < 0.01] = 0.0   # no return
    v = np.minimum(np.round(metres / 1000.0 * (2 ** 24 - 1)), 2 ** 24 - 1).astype(np.int64)
    rgb = np.stack([v & 255, (v >> 8) & 255, v >> 16], -1).astype(np.uint8)
    Image.fromarray(rgb, "RGB").save(path, compress_level=1)


def _topdown_png(path, g):
    bev = np.zeros((200, 200), dtype=np.uint8)
    bev[:, 80:120] = 128                       # drivable area
    for _ in range(int(g.integers(2, 6))):     # parked vehicles (grey 75 -> class 1)
        r, c = g.integers(10, 180, 2)
        bev[r:r + 10, c:c + 5] = 75
    r, c = g.integers(20, 170, 2)
    bev[r:r + 4, c:c + 4] = 255                # already-white pixels (-> class 2)
    Image.fromarray(np.repeat(bev[..., None], 3, -1), "RGB").save(path, compress_level=1)


def make_task(task_dir, frames, seed, hist=10, future=4):
    """Measurements for every frame; sensor images only for the frames CarlaDataset turns into
    samples, [hist, frames - future) (dataset/carla_dataset.py:291) — the others are never read."""
    g = np.random.default_rng(seed)
    for sub in [f"rgb_{c}" for c in CAMS] + [f"depth_{c}" for c in CAMS] + \
            ["topdown", "measurements", "parking_goal"]:
        os.makedirs(os.path.join(task_dir, sub), exist_ok=True)
    x0, y0, yaw0 = g.uniform(200, 300), g.uniform(-250, -150), g.uniform(-180, 180)
    goal = {"x": x0 + g.uniform(-4, 4), "y": y0 + g.uniform(-4, 4), "z": 0.3,
            "yaw": float(g.uniform(-180, 180))}
    with open(os.path.join(task_dir, "parking_goal", "0001.json"), "w") as f:
        json.dump(goal, f)
    for i in range(frames):
        name = f"{i:04d}"
        if hist <= i < frames - future:
            ig = np.random.default_rng([seed, i, 0])
            for c in CAMS:
                _camera_png(os.path.join(task_dir, f"rgb_{c}", name + ".png"), ig)
                _depth_png(os.path.join(task_dir, f"depth_{c}", name + ".png"), ig)
            _topdown_png(os.path.join(task_dir, "topdown", f"encoded_{name}.png"), ig)
        fg = np.random.default_rng([seed, i, 1])
        brake = float(fg.uniform(0, 1)) if fg.uniform() < 0.3 else 0.0
        m = {"x": x0 + 0.05 * i, "y": y0 - 0.03 * i, "z": 0.03, "pitch": float(fg.uniform(-1, 1)),
             "yaw": yaw0 + 0.5 * i, "roll": float(fg.uniform(-1, 1)),
             "speed": float(fg.uniform(0, 3)), "acc_x": float(fg.uniform(-2, 2)),
             "acc_y": float(fg.uniform(-2, 2)), "Throttle": float(fg.uniform(0, 1)),
             "Brake": brake, "Steer": float(fg.uniform(-1, 1)),
             "Reverse": bool(fg.uniform() < 0.3)}
        with open(os.path.join(task_dir, "measurements", name + ".json"), "w") as f:
            json.dump(m, f)


def make_dataset(root, frames=16, layout=None):
    """Write the mini dataset; returns the list of task directories written.
    layout: {town: {route: [task, ...]}}."""
    layout = layout or {TRAIN_TOWN: {"route_0": ["task_0", "task_1"], "route_1": ["task_0", "task_1"]},
                        VAL_TOWN: {"route_0": ["task_0"]}}
    tasks = []
    for town, routes in layout.items():
        for route, names in routes.items():
            for t in names:
                d = os.path.join(root, town, route, t)
                make_task(d, frames, _seed(f"{town}/{route}/{t}"))
                tasks.append(d)
    return tasks


def config(root, **kw):
    from tool.config import default_cfg
    return default_cfg(data_dir=root, training_map=TRAIN_TOWN, validation_map=VAL_TOWN, **kw)
