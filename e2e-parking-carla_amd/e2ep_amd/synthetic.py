"""Camera rig and synthetic batches for the ParkingModel hot path.

The rig restates the constant CARLA camera setup the reference trains on
(reference dataset/carla_dataset.py:206-270, data_generation/world.py:241-317):
four 400x300 FOV-100 cameras, centre-cropped to 256, with K adjusted by
tool/geometry.py:16-37 (update_intrinsics) and E = cam2pixel @ inverse(cam2veh) using
CARLA's Transform matrix convention (LibCarla Transform::GetMatrix, restated).

Synthetic batches follow SURVEY.md §8(d): every tensor is drawn from a CPU
torch.Generator seeded per call, so the same (B, seed) gives the same batch on any host.
The batch dict has exactly the reference schema (dataset/carla_dataset.py:379-423).
"""
import numpy as np
import torch

from .carla_math import Location, Rotation, Transform

# (x, y, z, pitch, yaw) in metres / degrees; order = front, left, right, rear
# (dataset/carla_dataset.py:209-230, 266-270)
CAMS_4 = [
    (1.5, 0.0, 1.5, 0.0, 0.0),
    (0.0, -0.8, 1.5, -40.0, -90.0),
    (0.0, 0.8, 1.5, -40.0, 90.0),
    (-2.2, 0.0, 1.5, -30.0, 180.0),
]
# C4 hi-res rig adds front-left / front-right
CAMS_6 = CAMS_4 + [
    (1.0, -0.8, 1.5, -20.0, -45.0),
    (1.0, 0.8, 1.5, -20.0, 45.0),
]

_CAM2PIXEL = np.array([[0, 1, 0, 0], [0, 0, -1, 0], [1, 0, 0, 0], [0, 0, 0, 1]], dtype=float)


def _carla_inverse_matrix(x, y, z, pitch, yaw, roll=0.0):
    t = Transform(Location(x, y, z), Rotation(pitch=pitch, yaw=yaw, roll=roll))
    return np.array(t.get_inverse_matrix())


def rig(n_cams=4, image=256, raw_w=400, raw_h=300, fov=100.0):
    """Return (K (N,3,3) f32, E (N,4,4) f32) for the reference rig cropped to `image`.

    For the hi-res 6-camera rig pass n_cams=6, image=512, raw_w=raw_h=512."""
    cams = CAMS_4 if n_cams == 4 else CAMS_6
    f = raw_w / (2 * np.tan(fov * np.pi / 360))
    k = torch.from_numpy(np.array([[f, 0, raw_w / 2], [0, f, raw_h / 2], [0, 0, 1]], dtype=float)).float()
    k = k.clone()
    k[0, 2] -= (raw_w - image) / 2
    k[1, 2] -= (raw_h - image) / 2
    K = k.unsqueeze(0).expand(len(cams), 3, 3).contiguous()
    E = torch.stack([torch.from_numpy(_CAM2PIXEL @ _carla_inverse_matrix(*c)).float() for c in cams])
    return K, E


def synthetic_batch(batch=8, n_cams=4, image=256, seed=0, bev=200, token_nums=204, hires=False):
    """A reference-schema batch (CPU tensors) of synthetic data, SURVEY.md §8(d)."""
    g = torch.Generator().manual_seed(seed)
    if hires:
        K, E = rig(6, 512, 512, 512)
        n_cams, image = 6, 512
    else:
        K, E = rig(n_cams, image)
    B = batch
    u = lambda *s: torch.rand(*s, generator=g)
    data = {
        "image": torch.randn(B, n_cams, 3, image, image, generator=g),
        "intrinsics": K.unsqueeze(0).expand(B, -1, -1, -1).contiguous(),
        "extrinsics": E.unsqueeze(0).expand(B, -1, -1, -1).contiguous(),
    }
    tp = torch.empty(B, 3)
    tp[:, :2] = u(B, 2) * 12.0 - 6.0
    tp[:, 2] = u(B) * 360.0 - 180.0
    data["target_point"] = tp
    em = torch.empty(B, 1, 3)
    em[..., 0] = u(B, 1) * 12.0
    em[..., 1:] = u(B, 1, 2) * 6.0 - 3.0
    data["ego_motion"] = em
    ctrl = torch.randint(0, token_nums - 4, (B, 12), generator=g)
    bos, eos, pad = token_nums - 3, token_nums - 2, token_nums - 1
    data["gt_control"] = torch.cat([torch.full((B, 1), bos), ctrl, torch.full((B, 1), eos),
                                    torch.full((B, 1), pad)], 1).long()
    data["segmentation"] = torch.randint(0, 3, (B, 1, bev, bev), generator=g).long()
    data["depth"] = u(B, n_cams, image, image) * 15.0
    data["gt_acc"] = u(B, 4) * 2 - 1
    data["gt_steer"] = u(B, 4) * 2 - 1
    data["gt_reverse"] = torch.randint(0, 2, (B, 4), generator=g).long()
    return data


def target_noise(batch, seed=0):
    """The (B,2) uniform draw that replaces torch.rand_like at model/parking_model.py:36."""
    return torch.rand(batch, 2, generator=torch.Generator().manual_seed(10_000 + seed))
