"""CarlaDataset and its helpers — drop-in for the reference's dataset/carla_dataset.py.

Same module path, class/function names, constructor arguments, sample schema and values as
the reference (dataset/carla_dataset.py:12-515), without its `carla`, `torchvision` and
`loguru` imports (none is part of this image):
  * CARLA Transform matrices come from e2ep_amd.carla_math (float64 restatement of LibCarla's
    convention, see there);
  * torchvision ToTensor + Normalize is restated as uint8 -> fp32 /255, minus mean, divided by
    std, in that order and in fp32 (what torchvision 0.14 computes);
  * logging goes through the standard `logging` module.
Decoding stays on the CPU with PIL exactly as the reference does: this is the reference data
path, and the parity anchor for the MI355X frame cache (dataset/frame_cache.py), which decodes
the same frames once into uint8 arrays and finishes the per-step arithmetic on the GPU.

Numerics note: the slot-drawing pixel arithmetic follows numpy 1.21, the reference's pinned
version (environment.yml:69), where np.float32 / Python float promotes to float64.
"""
import json
import logging
import os

import numpy as np
import torch
import torch.utils.data
from PIL import Image

from e2ep_amd.carla_math import Location, Rotation, Transform

log = logging.getLogger(__name__)

IMAGENET_MEAN = (0.485, 0.456, 0.406)
IMAGENET_STD = (0.229, 0.224, 0.225)
CAMERAS = ("front", "left", "right", "rear")
# camera mounts (dataset/carla_dataset.py:209-230): x, y, z [m], roll, pitch, yaw [deg]
CAMERA_MOUNTS = {
    "rgb_front": (1.5, 0.0, 1.5, 0.0, 0.0, 0.0),
    "rgb_left": (0.0, -0.8, 1.5, 0.0, -40.0, -90.0),
    "rgb_right": (0.0, 0.8, 1.5, 0.0, -40.0, 90.0),
    "rgb_rear": (-2.2, 0.0, 1.5, 0.0, -30.0, 180.0),
}
RAW_W, RAW_H, FOV = 400, 300, 100
CAM2PIXEL = np.array([[0, 1, 0, 0], [0, 0, -1, 0], [1, 0, 0, 0], [0, 0, 0, 1]], dtype=float)
DEPTH_WEIGHTS = np.array([1.0, 256.0, 65536.0])   # CARLA depth: R + 256 G + 65536 B
DEPTH_FAR = 1000.0                                  # metres at 2^24 - 1


def convert_veh_coord(x, y, z, ego_trans):
    """World point (x, y, z) -> ego-vehicle frame (dataset/carla_dataset.py:33-46)."""
    world2veh = np.array(ego_trans.get_inverse_matrix())
    return world2veh @ np.array([x, y, z, 1.0], dtype=float)


def convert_slot_coord(ego_trans, target_point):
    """Parking goal [x, y, yaw] in the world frame -> ego frame, yaw difference wrapped into
    [-180, 180] (dataset/carla_dataset.py:12-30)."""
    p = convert_veh_coord(target_point[0], target_point[1], 1.0, ego_trans)
    dyaw = target_point[2] - ego_trans.rotation.yaw
    if dyaw > 180:
        dyaw -= 360
    elif dyaw < -180:
        dyaw += 360
    return [p[0], p[1], dyaw]


def scale_and_crop_image(image, scale=1.0, crop=256):
    """PIL image -> nearest-neighbour resize by 1/scale -> centred crop x crop numpy array
    (dataset/carla_dataset.py:49-64)."""
    w, h = int(image.width // scale), int(image.height // scale)
    arr = np.asarray(image.resize((w, h), resample=Image.NEAREST))
    top, left = h // 2 - crop // 2, w // 2 - crop // 2
    return arr[top:top + crop, left:left + crop].copy()


def tokenize(throttle, brake, steer, reverse, token_nums=200):
    """Controls -> [throttle/brake, steer, reverse] tokens in [0, token_nums - 4]
    (dataset/carla_dataset.py:67-87)."""
    span = token_nums - 4
    half = span / 2
    acc = -brake if brake != 0.0 else throttle
    return [int(half * (acc + 1)), int((steer + 1) * half), int(reverse * span)]


def detokenize(token_list, token_nums=200):
    """Tokens -> [throttle, brake, steer, reverse] (dataset/carla_dataset.py:90-111)."""
    half = float((token_nums - 4) / 2)
    acc = token_list[0] / half - 1
    throttle, brake = (acc, 0.0) if token_list[0] > half else (0.0, -acc)
    return [throttle, brake, token_list[1] / half - 1, bool(token_list[2] > half)]


def load_rgb(image_path, crop):
    """The cropped camera PNG as uint8 RGB (crop, crop, 3) — ProcessImage's crop."""
    return scale_and_crop_image(Image.open(image_path).convert("RGB"), scale=1.0, crop=crop)


def load_depth_rgb(depth_image_path, crop):
    """The cropped CARLA depth PNG as uint8 RGB (crop, crop, 3) — get_depth's input."""
    return scale_and_crop_image(Image.open(depth_image_path).convert("RGB"), scale=1.0, crop=crop)


def depth_from_rgb(rgb):
    """uint8 CARLA depth RGB -> float64 metres: (R + 256 G + 65536 B) / (2^24 - 1) * 1000.
    The weighted sum is an exact integer in float64, so this equals the reference's
    float32-cast np.dot (dataset/carla_dataset.py:125-129) bit for bit."""
    d = np.asarray(rgb, dtype=np.float64) @ DEPTH_WEIGHTS
    d /= (1 << 24) - 1
    return DEPTH_FAR * d


def get_depth(depth_image_path, crop):
    """CARLA depth PNG -> (1, crop, crop) float64 metres (dataset/carla_dataset.py:114-131)."""
    return torch.from_numpy(depth_from_rgb(load_depth_rgb(depth_image_path, crop))).unsqueeze(0)


def update_intrinsics(intrinsics, top_crop=0.0, left_crop=0.0, scale_width=1.0, scale_height=1.0):
    """Pinhole K after scaling then cropping (dataset/carla_dataset.py:134-145)."""
    k = intrinsics.clone()
    k[0, 0] *= scale_width
    k[0, 2] *= scale_width
    k[1, 1] *= scale_height
    k[1, 2] *= scale_height
    k[0, 2] -= left_crop
    k[1, 2] -= top_crop
    return k


def add_raw_control(data, throttle_brake, steer, reverse):
    """Append one frame's raw controls (dataset/carla_dataset.py:148-154)."""
    throttle_brake.append(-data["Brake"] if data["Brake"] != 0.0 else data["Throttle"])
    steer.append(data["Steer"])
    reverse.append(int(data["Reverse"]))


def camera_rig(image_crop):
    """(intrinsics (4,3,3) f32 expanded view, extrinsics (4,4,4) f32) of the four dataset
    cameras (dataset/carla_dataset.py:206-270)."""
    f = RAW_W / (2 * np.tan(FOV * np.pi / 360))
    k0 = np.array([[f, 0, RAW_W / 2], [0, f, RAW_H / 2], [0, 0, 1]], dtype=float)
    k = update_intrinsics(torch.from_numpy(k0).float(), (RAW_H - image_crop) / 2,
                          (RAW_W - image_crop) / 2, scale_width=1, scale_height=1)
    veh2cam = {}
    for cam, (x, y, z, roll, pitch, yaw) in CAMERA_MOUNTS.items():
        cam2veh = Transform(Location(x=x, y=y, z=z), Rotation(yaw=yaw, pitch=pitch, roll=roll))
        veh2cam[cam] = CAM2PIXEL @ np.array(cam2veh.get_inverse_matrix())
    ext = torch.cat([torch.from_numpy(veh2cam["rgb_" + c]).float().unsqueeze(0) for c in CAMERAS], 0)
    return k.unsqueeze(0).expand(4, 3, 3), ext, veh2cam


class CarlaDataset(torch.utils.data.Dataset):
    """One sample per frame of every parking task under <root>/<town>/<route>/<task>/, frames
    [hist_frame_nums, total - future_frame_nums) (dataset/carla_dataset.py:157-423)."""

    def __init__(self, root_dir, is_train, config):
        super().__init__()
        self.cfg = config
        self.BOS_token = self.cfg.token_nums - 3
        self.EOS_token = self.BOS_token + 1
        self.PAD_token = self.EOS_token + 1
        self.root_dir = root_dir
        self.is_train = is_train
        self.image_crop = self.cfg.image_crop
        self.intrinsic = None
        self.veh2cam_dict = {}
        self.extrinsic = None
        self.image_process = ProcessImage(self.image_crop)
        self.semantic_process = ProcessSemantic(self.cfg)
        self.init_camera_config()
        for name in ("front", "left", "right", "rear", "front_depth", "left_depth", "right_depth",
                     "rear_depth", "control", "velocity", "acc_x", "acc_y", "throttle_brake",
                     "steer", "reverse", "target_point", "topdown"):
            setattr(self, name, [])
        self.get_data()

    def init_camera_config(self):
        self.intrinsic, self.extrinsic, self.veh2cam_dict = camera_rig(self.image_crop)

    def task_dirs(self):
        """Task directories in os.listdir order — the reference's sample order."""
        town = self.cfg.training_map if self.is_train == 1 else self.cfg.validation_map
        town_dir = os.path.join(self.root_dir, town)
        return [os.path.join(town_dir, route, task)
                for route in os.listdir(town_dir)
                for task in os.listdir(os.path.join(town_dir, route))]

    def get_data(self):
        hist, future = self.cfg.hist_frame_nums, self.cfg.future_frame_nums
        for task in self.task_dirs():
            cache = {}

            def measurement(i):
                if i not in cache:
                    with open(task + f"/measurements/{str(i).zfill(4)}.json", "r") as f:
                        cache[i] = json.load(f)
                return cache[i]

            with open(task + "/parking_goal/0001.json", "r") as f:
                goal = json.load(f)
            total = len(os.listdir(task + "/measurements/"))
            for frame in range(hist, total - future):
                name = f"{str(frame).zfill(4)}.png"
                for cam in CAMERAS:
                    getattr(self, cam).append(task + f"/rgb_{cam}/" + name)
                    getattr(self, cam + "_depth").append(task + f"/depth_{cam}/" + name)
                self.topdown.append(task + "/topdown/encoded_" + name)
                m = measurement(frame)
                ego = Transform(Location(x=m["x"], y=m["y"], z=m["z"]),
                                Rotation(yaw=m["yaw"], pitch=m["pitch"], roll=m["roll"]))
                self.velocity.append(m["speed"])
                self.acc_x.append(m["acc_x"])
                self.acc_y.append(m["acc_y"])
                tokens, acc, steer, rev = [self.BOS_token], [], [], []
                for i in range(future):
                    n = measurement(frame + 1 + i)
                    tokens += tokenize(n["Throttle"], n["Brake"], n["Steer"], n["Reverse"],
                                       self.cfg.token_nums)
                    add_raw_control(n, acc, steer, rev)
                self.control.append(tokens + [self.EOS_token, self.PAD_token])
                self.throttle_brake.append(acc)
                self.steer.append(steer)
                self.reverse.append(rev)
                self.target_point.append(convert_slot_coord(ego, [goal["x"], goal["y"], goal["yaw"]]))

        for name in ("front", "left", "right", "rear", "front_depth", "left_depth", "right_depth",
                     "rear_depth", "topdown"):
            setattr(self, name, np.array(getattr(self, name), dtype=str))
        for name, dt in (("velocity", np.float32), ("acc_x", np.float32), ("acc_y", np.float32),
                         ("control", np.int64), ("throttle_brake", np.float32),
                         ("steer", np.float32), ("reverse", np.int64), ("target_point", np.float32)):
            setattr(self, name, np.array(getattr(self, name)).astype(dt))
        log.info("Preloaded %d sequences", len(self.front))

    def __len__(self):
        return len(self.front)

    def __getitem__(self, index):
        images = [self.image_process(getattr(self, c)[index])[0] for c in CAMERAS]
        depths = [get_depth(getattr(self, c + "_depth")[index], self.image_crop) for c in CAMERAS]
        seg = self.semantic_process(self.topdown[index], scale=0.5, crop=200,
                                    target_slot=self.target_point[index])
        return {
            "image": torch.cat(images, dim=0),
            "depth": torch.cat(depths, dim=0),
            "extrinsics": self.extrinsic,
            "intrinsics": self.intrinsic,
            "target_point": torch.from_numpy(self.target_point[index]),
            "ego_motion": torch.from_numpy(np.column_stack(
                (self.velocity[index], self.acc_x[index], self.acc_y[index]))),
            "segmentation": torch.from_numpy(seg).long().unsqueeze(0),
            "gt_control": torch.from_numpy(self.control[index]),
            "gt_acc": torch.from_numpy(self.throttle_brake[index]),
            "gt_steer": torch.from_numpy(self.steer[index]),
            "gt_reverse": torch.from_numpy(self.reverse[index]),
        }


# the parking slot footprint in BEV pixels around its centre (dataset/carla_dataset.py:473-476)
_SLOT_GRID = np.array([[x, y, 1, 1] for x in range(-27, 28) for y in range(-15, 16)], dtype=int).T


class ProcessSemantic:
    """Topdown BEV PNG -> (200, 200) float64 classes {0 background, 1 vehicle, 2 target slot}
    in the LSS orientation (dataset/carla_dataset.py:426-491)."""

    def __init__(self, cfg):
        self.cfg = cfg

    def __call__(self, image, scale, crop, target_slot):
        if not isinstance(image, Image.Image):
            image = Image.open(image)
        bev = self.draw_target_slot(scale_and_crop_image(image.convert("L"), scale, crop),
                                    target_slot)
        classes = np.zeros(bev.shape)
        classes[bev == 75] = 1
        classes[bev == 255] = 2
        return classes[::-1].copy()

    def draw_target_slot(self, image, target_slot):
        size = image.shape[0]
        px = float(target_slot[0]) / self.cfg.bev_x_bound[2]
        py = float(target_slot[1]) / self.cfg.bev_y_bound[2]
        centre = np.array([size / 2 - px, size / 2 + py], dtype=int)
        rot = np.array(Transform(Location(), Rotation(yaw=float(-target_slot[2]))).get_matrix())
        pts = (rot @ _SLOT_GRID)[0:2].astype(int)
        pts[0] += centre[0]
        pts[1] += centre[1]
        image[tuple(pts)] = 255
        return image


_MEAN = torch.tensor(IMAGENET_MEAN).view(3, 1, 1)
_STD = torch.tensor(IMAGENET_STD).view(3, 1, 1)


def normalise_image(rgb):
    """uint8 (H, W, 3) -> fp32 (3, H, W): /255, minus ImageNet mean, over std (torchvision
    ToTensor + Normalize, dataset/carla_dataset.py:498-502)."""
    t = torch.from_numpy(np.ascontiguousarray(np.asarray(rgb).transpose(2, 0, 1))).float().div(255)
    return t.sub_(_MEAN).div_(_STD)


class ProcessImage:
    """Camera frame (path, PIL image, or a CARLA sensor image with BGRA `raw_data`) ->
    ((1, 3, crop, crop) normalised fp32, (crop, crop, 3) uint8 crop)
    (dataset/carla_dataset.py:494-515)."""

    def __init__(self, crop):
        self.crop = crop
        self.normalise_image = normalise_image

    def __call__(self, image):
        if hasattr(image, "raw_data"):
            bgra = np.frombuffer(bytes(image.raw_data), dtype=np.uint8)
            bgra = bgra.reshape(image.height, image.width, 4)
            image = Image.fromarray(np.ascontiguousarray(bgra[:, :, 2::-1]))
        elif not isinstance(image, Image.Image):
            image = Image.open(image).convert("RGB")
        else:
            image = image.convert("RGB")
        crop = scale_and_crop_image(image, scale=1.0, crop=self.crop)
        return self.normalise_image(np.array(crop)).unsqueeze(0), crop
