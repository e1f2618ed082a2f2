"""How many pixels the single-layer glass rule can change.

The reference draws glass last with depth writes on and blends every front-facing
glass face a pixel's ray crosses, in mesh order (render.js:82-86, sdf.cpp:284,337);
the build blends the first glass face over the first opaque surface behind it.
The two agree wherever a ray crosses at most one glass face.  This counts, per
frame, the pixels whose ray crosses 0, 1, 2, 3+ glass faces before the opaque
hit (oracle.Oracle.glass_layers: the primary walk's glass entries).
usage: python tools/glass_layers.py [--config C3] [--cams K0,K1,K2]
"""
import argparse
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="C3")
    ap.add_argument("--cams", default="K0,K1,K2")
    ap.add_argument("--threads", type=int, default=0)
    args = ap.parse_args()
    import numpy as np

    import oracle
    import voxmap_amd as vx
    from voxmap_amd import presets
    c = presets.CONFIGS[args.config]
    field = vx.field_build(presets.scene_grid(c["scene"]))
    O = oracle.Oracle(field, np.zeros((16, 16, 4), np.uint8))
    out = {}
    for cam in args.cams.split(","):
        fr = presets.camera_frame(cam, c["w"], c["h"])
        n = O.glass_layers(fr.params, c["w"], c["h"], threads=args.threads)
        hist = np.bincount(n.ravel(), minlength=4)
        out[cam] = {"pixels": int(n.size), "glass_0": int(hist[0]), "glass_1": int(hist[1]),
                    "glass_2": int(hist[2]), "glass_3plus": int(hist[3:].sum()),
                    "share_2plus": float(hist[2:].sum() / n.size)}
    print(json.dumps({"config": args.config, "scene": c["scene"], "frames": out}, indent=1))


if __name__ == "__main__":
    main()
