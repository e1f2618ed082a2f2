"""Sun exit table probe (DESIGN.md §3 "Sun exit tables"): one BASELINE
workload rendered with the cone + orthant tables (default), the orthant tables
only (VX_FLAG_NO_CONE) and none (VX_FLAG_NO_EXIT): frames must be identical;
prints the shadow fetch counts (the steps this build takes against the
reference's own step count) and the one-stream launch times.

usage: python tools/exit_probe.py [--config C3] [--flags 48]
"""
from __future__ import annotations

import argparse
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="C3")
    ap.add_argument("--flags", default="0,48")
    ap.add_argument("--frames", type=int, default=20)
    args = ap.parse_args()
    import numpy as np
    import torch

    import voxmap_amd as vx
    from voxmap_amd import presets, scenes
    cfg = presets.CONFIGS[args.config]
    grid = presets.scene_grid(cfg["scene"])
    Z, Y, X = grid.shape
    W, H = cfg["w"], cfg["h"]
    up = 3.0 if cfg["scene"] == "s_up3" else 1.0
    samples = cfg.get("samples", 1)
    sc = vx.Scene(map_bytes=grid.tobytes(), map_format=vx.FORMAT_GRID, noise_path=scenes.NOISE_PATH,
                  dims=(X, Y, Z), device=0)
    out = torch.empty(W * H * 4, dtype=torch.uint8, device="cuda")
    st = torch.cuda.Stream()
    torch.cuda.set_stream(st)
    for flags in [int(f) for f in args.flags.split(",")]:
        res = {}
        for tag, fl in (("exit", flags), ("orthant", flags | vx.FLAG_NO_CONE), ("no_exit", flags | vx.FLAG_NO_EXIT)):
            fr = presets.camera_frame(cfg["camera"], W, H, scale=up, flags=fl, shadow_samples=samples,
                                      sun_radius=0.03 if samples > 1 else 0.0)
            s = sc.render_device(fr, out.data_ptr(), pixel_format=vx.PIXEL_RGBA8, stream=st.cuda_stream,
                                 stats=True).as_dict()
            torch.cuda.synchronize()
            img = out.cpu().numpy().copy()
            for _ in range(5):
                sc.render_device(fr, out.data_ptr(), pixel_format=vx.PIXEL_RGBA8, stream=st.cuda_stream)
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(args.frames):
                sc.render_device(fr, out.data_ptr(), pixel_format=vx.PIXEL_RGBA8, stream=st.cuda_stream)
            e1.record()
            torch.cuda.synchronize()
            res[tag] = (img, s, e0.elapsed_time(e1) / args.frames)
        same = bool(np.array_equal(res["exit"][0], res["no_exit"][0]) and
                    np.array_equal(res["orthant"][0], res["no_exit"][0]))
        print(json.dumps({"config": args.config, "flags": flags, "frames_identical": same,
                          "shadow_rays": res["exit"][1]["shadow_rays"],
                          "shadow_fetches_exit": res["exit"][1]["shadow_fetches"],
                          "shadow_fetches_orthant": res["orthant"][1]["shadow_fetches"],
                          "shadow_fetches_no_exit": res["no_exit"][1]["shadow_fetches"],
                          "ms_exit": round(res["exit"][2], 4), "ms_orthant": round(res["orthant"][2], 4),
                          "ms_no_exit": round(res["no_exit"][2], 4)}),
              flush=True)
        if not same:
            sys.exit(1)
    sc.close()


if __name__ == "__main__":
    main()
