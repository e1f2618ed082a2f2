"""GPU time of the frame's cone copy with and without the sun doom table
(vx_prepare_sun build_ms; DESIGN.md §3 "Doom table"), per bench scene.
usage: python tools/doom_build_time.py [--out profiles/r06_doom_build.json]"""
import argparse
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--out", default=None)
    args = ap.parse_args()
    import voxmap_amd as vx
    from voxmap_amd import presets, scenes
    res = {}
    for cfg in ("C3", "C5"):
        c = presets.CONFIGS[cfg]
        grid = presets.scene_grid(c["scene"])
        Z, Y, X = grid.shape
        sc = vx.Scene(map_bytes=grid.tobytes(), map_format=vx.FORMAT_GRID, noise_path=scenes.NOISE_PATH,
                      dims=(X, Y, Z), device=0)
        scale = 3.0 if c["scene"] == "s_up3" else 1.0
        n = 16                            # soft shadows: the frames that read the doom table
        r = {}
        for name, fl in (("no_doom", vx.FLAG_NO_DOOM), ("doom", 0), ("no_doom_again", vx.FLAG_NO_DOOM),
                         ("doom_again", 0)):
            fr = presets.camera_frame(c["camera"], 64, 64, scale=scale, flags=48 | fl, shadow_samples=n,
                                      sun_radius=0.03 if n else 0.0)
            # three slots' worth of distinct builds: evict by alternating windows
            r[name] = sc.prepare_sun(fr)
        sc.close()
        res[cfg] = {"dims": [X, Y, Z], "builds": r}
        print(cfg, json.dumps(res[cfg]), flush=True)
    if args.out:
        json.dump(res, open(args.out, "w"), indent=1)


if __name__ == "__main__":
    main()
