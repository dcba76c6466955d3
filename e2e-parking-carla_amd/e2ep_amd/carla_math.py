"""The CARLA transform arithmetic the reference's dataset uses, without the `carla` package.

The reference builds camera extrinsics, converts the parking goal into the ego frame and
rotates the drawn target slot with carla.Transform(Location, Rotation).get_matrix() /
get_inverse_matrix() (dataset/carla_dataset.py:32-46,254-270,476-488).  `carla` (0.9.11) is
a simulator client that is not part of this image; its Transform matrix convention
(LibCarla Transform::GetMatrix / GetInverseMatrix, degrees -> radians, yaw/pitch/roll) is
restated here in float64 — CARLA evaluates it in float32, so results can differ from a live
CARLA client in the last float32 bits (unpinned).
"""
import math

import numpy as np


class Location:
    def __init__(self, x=0.0, y=0.0, z=0.0):
        self.x, self.y, self.z = float(x), float(y), float(z)


class Rotation:
    def __init__(self, pitch=0.0, yaw=0.0, roll=0.0):
        self.pitch, self.yaw, self.roll = float(pitch), float(yaw), float(roll)


class Transform:
    def __init__(self, location=None, rotation=None):
        self.location = location if location is not None else Location()
        self.rotation = rotation if rotation is not None else Rotation()

    def _rot(self):
        cy, sy = math.cos(math.radians(self.rotation.yaw)), math.sin(math.radians(self.rotation.yaw))
        cp, sp = math.cos(math.radians(self.rotation.pitch)), math.sin(math.radians(self.rotation.pitch))
        cr, sr = math.cos(math.radians(self.rotation.roll)), math.sin(math.radians(self.rotation.roll))
        return np.array([[cp * cy, cy * sp * sr - sy * cr, -cy * sp * cr - sy * sr],
                         [cp * sy, sy * sp * sr + cy * cr, -sy * sp * cr + cy * sr],
                         [sp, -cp * sr, cp * cr]])

    def get_matrix(self):
        m = np.eye(4)
        m[:3, :3] = self._rot()
        m[:3, 3] = [self.location.x, self.location.y, self.location.z]
        return m.tolist()

    def get_inverse_matrix(self):
        r = self._rot()
        m = np.eye(4)
        m[:3, :3] = r.T
        m[:3, 3] = -r.T @ np.array([self.location.x, self.location.y, self.location.z])
        return m.tolist()
