"""Where the single glass layer and the reference's draw-order blend differ
(VERDICT r03 item 2): per C3 frame of S-proc and the stacked-glass
fixture S-glass, the pixels whose ray crosses 0 / 1 / 2 / 3+ front-facing panes
before the opaque surface, and the pixels whose fp32 RGBA (and RGBA8) differ
between the oracle's single layer and its VX_FLAG_GLASS_ORDER restatement
(render.js:82-91: glass quads in vertex.bin order, LESS + depth writes, SRC_ALPHA).
usage: python tools/glass_order_probe.py [--out profiles/r04_glass_order.json]"""
import argparse
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--out", default=None)
    ap.add_argument("--flags", type=int, default=48)
    args = ap.parse_args()
    import numpy as np

    import oracle
    import voxmap_amd as vx
    from voxmap_amd import presets, scenes
    noise = scenes.real_noise()
    res = {}
    for scene in ("s_proc", "s_glass"):
        field = vx.field_build(presets.scene_grid(scene))
        O = oracle.Oracle(field, noise, exit=True)
        for cam in ("K0", "K1", "K2"):
            fa = presets.camera_frame(cam, 3840, 2160, flags=args.flags)
            fb = presets.camera_frame(cam, 3840, 2160, flags=args.flags | vx.FLAG_GLASS_ORDER)
            a, _ = O.render(fa.params, 3840, 2160)
            b, _ = O.render(fb.params, 3840, 2160)
            n = O.glass_layers(fa.params, 3840, 2160)
            hist = np.bincount(n.ravel(), minlength=4)
            d = np.any(a.view(np.uint32) != b.view(np.uint32), axis=2)
            q = lambda im: np.floor(np.clip(im, 0, 1) * 255 + 0.5).astype(np.uint8)
            res[f"{scene}:{cam}"] = {"panes_0": int(hist[0]), "panes_1": int(hist[1]), "panes_2": int(hist[2]),
                                     "panes_3plus": int(hist[3:].sum()), "differ_fp32": int(d.sum()),
                                     "differ_rgba8": int(np.any(q(a) != q(b), axis=2).sum()),
                                     "differ_with_fewer_than_2_panes": int((d & (n < 2)).sum())}
            print(scene, cam, res[f"{scene}:{cam}"], flush=True)
    out = {"what": "oracle C3 frames (3840x2160, flags %d), single glass layer vs VX_FLAG_GLASS_ORDER" % args.flags,
           "frames": res}
    if args.out:
        json.dump(out, open(args.out, "w"), indent=1)


if __name__ == "__main__":
    main()
