"""Named, replayable benchmark / parity presets.

Cameras follow map.js:19-31 and :367 (orbit subject ``sbj``, rotation ``rot``;
orbit radius = sbj.z).  The sun uses hour = 1.0 (map.js:399-402), time 123 s.
Each sun component is non-zero, which keeps march() away from its
0*inf = NaN edge (render.frag:94-105).
"""
from __future__ import annotations

import math

from . import scenes
from .renderer import make_frame

# K0: the reference's default view after one frame of controls.rot/100 (map.js:20,24,31,367)
CAMERAS = {
    "K0": {"sbj": (381.5, 128.1, 128.0), "rot": (1e-4, 0.0, -0.002)},
    "K1": {"sbj": (381.5, 128.1, 40.0), "rot": (1.1, 0.0, 0.6)},      # oblique
    "K2": {"sbj": (0.0, 128.1, 12.0), "rot": (1.45, 0.0, -math.pi / 2)},  # grazing, from outside x=0 looking +x
}
SUN_HOUR = 1.0
TIME = 123.0

# BASELINE.json configs[0..4]
CONFIGS = {
    "C1": {"w": 256, "h": 256, "scene": "s_proc", "camera": "K0", "note": "primary-ray plumbing; host scalar"},
    "C2": {"w": 1920, "h": 1080, "scene": "s_proc", "camera": "K1", "note": "primary + shadow, 1 GPU"},
    "C3": {"w": 3840, "h": 2160, "scene": "s_proc", "camera": "K1", "note": "full v1 shading, 1 GPU"},
    "C4": {"w": 7680, "h": 4320, "scene": "s_proc", "camera": "K1", "note": "tiled across GPUs + RCCL gather"},
    "C5": {"w": 3840, "h": 2160, "scene": "s_up3", "camera": "K1", "samples": 16,
           "note": "3^3-upscaled field, 16-sample soft shadows"},
}


def camera_frame(name: str, w: int, h: int, scale: float = 1.0, **kw):
    """Frame for camera ``name``; ``scale`` multiplies the subject position (C5's 3x field)."""
    cam = CAMERAS[name]
    sbj = tuple(v * scale for v in cam["sbj"])
    kw.setdefault("hour", SUN_HOUR)
    kw.setdefault("time", TIME)
    return make_frame(sbj, cam["rot"], w, h, **kw)


def scene_grid(name: str, seed: int = 1):
    if name == "s_proc":
        return scenes.s_proc(seed)
    if name == "s_glass":
        return scenes.s_glass(seed)
    if name == "s_campus":
        return scenes.s_campus()
    if name == "s_up3":
        return scenes.upsample3(scenes.s_proc(seed))
    raise KeyError(name)


def sun_dir(hour: float = SUN_HOUR):
    return (math.sin(hour) * math.sqrt(0.75), math.sin(hour) * math.sqrt(0.25), abs(math.cos(hour)))
