"""Which pixels the GL blend stage changes (DESIGN.md §5 "The blend stage",
VERDICT r05 item 1): per C3 frame (3840x2160) of S-proc and S-glass, cameras
K0-K2, the oracle's frame with the RGBA8 canvas blend (clamped src/dst/alpha, dst
read back as unorm8 before every pane: blend_canvas) against the round-5 fp32
blend (the oracle-only diagnostic VXO_FLAG_BLEND_FLOAT).  Counts glass pixels,
pixels whose fp32 RGBA differs, whose RGBA8 differs, and by how many LSB.
usage: python tools/blend_probe.py [--flags 48] [--out profiles/r06_blend_probe.json]"""
import argparse
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

BLEND_FLOAT = 0x10000   # oracle/vxo.h VXO_FLAG_BLEND_FLOAT


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--out", default=None)
    ap.add_argument("--flags", type=int, nargs="+", default=[48, 0])
    ap.add_argument("--w", type=int, default=3840)
    ap.add_argument("--h", type=int, default=2160)
    args = ap.parse_args()
    import numpy as np

    import oracle
    import voxmap_amd as vx
    from voxmap_amd import presets, scenes
    noise = scenes.real_noise()
    q = lambda im: np.floor(np.clip(im, 0, 1) * np.float32(255) + np.float32(0.5)).astype(np.int32)
    res = {}
    for scene in ("s_proc", "s_glass"):
        field = vx.field_build(presets.scene_grid(scene))
        O = oracle.Oracle(field, noise, exit=True)
        for fl in args.flags:
            for cam in ("K0", "K1", "K2"):
                fa = presets.camera_frame(cam, args.w, args.h, flags=fl)
                fb = presets.camera_frame(cam, args.w, args.h, flags=fl | BLEND_FLOAT)
                a, st = O.render(fa.params, args.w, args.h)
                b, _ = O.render(fb.params, args.w, args.h)
                d = np.any(a.view(np.uint32) != b.view(np.uint32), axis=2)
                dq = np.abs(q(a) - q(b)).max(axis=2)
                r = {"glass_px": int(st.glass_px), "differ_fp32": int(d.sum()),
                     "differ_rgba8": int((dq > 0).sum()), "differ_rgba8_over_1_lsb": int((dq > 1).sum()),
                     "max_lsb": int(dq.max())}
                res[f"{scene}:{cam}:flags{fl}"] = r
                print(scene, cam, fl, r, flush=True)
    out = {"what": "oracle frames %dx%d, RGBA8 canvas blend vs the round-5 fp32 blend" % (args.w, args.h),
           "frames": res}
    if args.out:
        json.dump(out, open(args.out, "w"), indent=1)


if __name__ == "__main__":
    main()
