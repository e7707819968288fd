"""Camera with the reference's view-projection (ref: apps/frontend/src/graphics-core/Camera.ts).

``GetViewProjectionMatrix`` = P · inverse(T · R) with ``R = fromQuat(fromEuler(pitch,
yaw, roll, "yxz"))`` (Camera.ts:47-64) and ``P = perspective(60°, W/H, 0.1, 1000)``
(Camera.ts:19-45,165-168); the renderer uploads ``invert(VP)`` (Renderer_TEST.ts:172).
"""
from __future__ import annotations

import math

import numpy as np

from . import wgpu_math as wm


class Camera:
    def __init__(self, width: int, height: int, location=(0.0, 0.0, 1.0), roll_deg=0.0, pitch_deg=0.0,
                 yaw_deg=0.0, fov_deg=60.0, near=0.1, far=1000.0):
        self.location = np.asarray(location, dtype=np.float32).copy()
        self.roll = roll_deg * math.pi / 180.0
        self.pitch = pitch_deg * math.pi / 180.0
        self.yaw = yaw_deg * math.pi / 180.0
        self.aspect = width / height
        self.fov = fov_deg * math.pi / 180.0
        self.near = near
        self.far = far
        self.projection = wm.mat4_perspective(self.fov, self.aspect, self.near, self.far)

    # Camera.ts:149-156
    def set_location(self, x, y, z):
        self.location[:] = (x, y, z)

    def set_yaw(self, deg):
        self.yaw = math.fmod(deg * math.pi / 180.0, 2 * math.pi)

    def set_pitch(self, deg):
        self.pitch = min(math.pi, max(-math.pi, deg * math.pi / 180.0))

    # Camera.ts:116-130 (degrees in, radians stored; JS % is fmod)
    def add_pitch(self, deg):
        self.pitch = min(math.pi / 2, max(-math.pi / 2, self.pitch + deg * math.pi / 180.0))

    def add_yaw(self, deg):
        self.yaw = math.fmod(self.yaw + deg * math.pi / 180.0, 2 * math.pi)

    # Camera.ts:139-146: the Float32Array location, component by component
    def add_location_offset(self, o):
        o = np.asarray(o, dtype=np.float32)
        for i in range(3):
            self.location[i] = np.float32(float(self.location[i]) + float(o[i]))

    # Camera.ts:157-163
    def set_aspect_ratio(self, width, height):
        self.aspect = width / height
        self.projection = wm.mat4_perspective(self.fov, self.aspect, self.near, self.far)

    # Camera.ts:66-81
    def forward_vector(self) -> np.ndarray:
        q = wm.quat_from_euler(self.pitch, self.yaw, self.roll, "yxz")
        return wm.vec3_normalize(wm.vec3_transform_quat(np.array([0, 0, -1], np.float32), q))

    def right_vector(self) -> np.ndarray:
        return wm.vec3_cross(self.forward_vector(), np.array([0, 1, 0], np.float32))

    def view_matrix(self) -> np.ndarray:
        t = wm.mat4_translation(self.location)
        r = wm.mat4_from_quat(wm.quat_from_euler(self.pitch, self.yaw, self.roll, "yxz"))
        return wm.mat4_invert(wm.mat4_multiply(t, r))

    def view_projection(self) -> np.ndarray:
        return wm.mat4_multiply(self.projection, self.view_matrix())

    def view_projection_inverse(self) -> np.ndarray:
        return wm.mat4_invert(self.view_projection())
