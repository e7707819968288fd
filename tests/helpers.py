"""Shared helpers for the parity tests."""
import numpy as np

from pathtracerdemo_amd.scene.camera import Camera


def uniform_for(cs, W, H, frame=1, location=(0.0, 0.0, 6.0), yaw=0.0, pitch=0.0):
    cam = Camera(W, H)
    cam.set_location(*location)
    if yaw:
        cam.set_yaw(yaw)
    if pitch:
        cam.set_pitch(pitch)
    return cs.uniform(W, H, cam.view_projection_inverse(), cam.location, frame)


def rel_l2(a, b):
    a = np.asarray(a, np.float64)
    b = np.asarray(b, np.float64)
    finite = np.isfinite(a) & np.isfinite(b)
    num = np.sqrt(((a - b)[finite] ** 2).sum())
    den = np.sqrt((b[finite] ** 2).sum())
    return float(num / den) if den > 0 else float(num)
