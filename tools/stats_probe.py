"""Work counters of one frame per bench config, with the lane utilisations
they imply (STATS instantiation of k_render, MI355X):

  primary lane util = primary_fetches / (64 * primary_wave_iters)
  march lane util   = shadow_fetches  / (64 * march_wave_iters)

usage: python tools/stats_probe.py [C3 C5 ...]  (default: C3 C5)
"""
from __future__ import annotations

import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    import torch

    import voxmap_amd as vx
    from voxmap_amd import presets, scenes
    torch.cuda.set_device(0)
    for name in sys.argv[1:] or ["C3", "C5"]:
        cfg = presets.CONFIGS[name]
        grid = presets.scene_grid(cfg["scene"])
        Z, Y, X = grid.shape
        up = 3.0 if cfg["scene"] == "s_up3" else 1.0
        scene = vx.Scene(map_bytes=grid.tobytes(), map_format=vx.FORMAT_GRID, noise_path=scenes.NOISE_PATH,
                         dims=(X, Y, Z), device=0)
        samples = cfg.get("samples", 1)
        for flags in (0, vx.FLAG_FULL_QUALITY):
            fr = presets.camera_frame(cfg["camera"], cfg["w"], cfg["h"], scale=up, flags=flags,
                                      shadow_samples=samples, sun_radius=0.03 if samples > 1 else 0.0)
            out = torch.empty(cfg["w"] * cfg["h"] * 4, dtype=torch.uint8, device="cuda")
            st = scene.render_device(fr, out.data_ptr(), pixel_format=vx.PIXEL_RGBA8, stats=True)
            torch.cuda.synchronize()
            d = st.as_dict() if hasattr(st, "as_dict") else dict(st)
            d["config"], d["flags"] = name, flags
            d["primary_lane_util"] = d["primary_fetches"] / max(1, 64 * d["primary_wave_iters"])
            d["march_lane_util"] = d["shadow_fetches"] / max(1, 64 * d["march_wave_iters"])
            d["primary_steps_per_px"] = d["primary_fetches"] / max(1, d["pixels"])
            d["shadow_steps_per_ray"] = d["shadow_fetches"] / max(1, d["shadow_rays"])
            print(json.dumps(d), flush=True)
        scene.close()
        del grid


if __name__ == "__main__":
    main()
