"""Where the doom table for the hard shadow (ab/doom_hard.so, VX_AB_DOOM_HARD)
changes a frame: small-scene frames against the oracle (which renders the same
pixels with or without the table), and the C3 K1 frame against NO_DOOM.
usage: VOXMAP_LIB=ab/doom_hard.so python tools/doom_hard_probe.py"""
import math
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    import oracle
    import voxmap_amd as vx
    from voxmap_amd import presets, scenes
    noise = np.frombuffer(vx.decode(open(scenes.NOISE_PATH, "rb").read(), vx.FORMAT_BIN_GZ), np.uint8).reshape(1024, 1024, 4).copy()
    dims = (96, 64, 40)
    field = vx.field_build(scenes.small_proc(31, dims=dims, n_boxes=30, n_glass=5))
    sc = vx.Scene(map_bytes=field.tobytes(), map_format=vx.FORMAT_BIN, noise_bytes=noise.tobytes(),
                  noise_format=vx.FORMAT_BIN, dims=dims, device=0)
    o = oracle.Oracle(sc.read_field(), noise, exit=True)
    for el, az in [(33, 30), (40, 120), (60, 210), (20, 300), (15, 45)]:
        e, a = math.radians(el), math.radians(az)
        sun = (math.cos(e) * math.cos(a), math.cos(e) * math.sin(a), math.sin(e))
        for fl in (48, 0, 1):
            fr = vx.make_frame((48.0, 32.0, 36.0), (1.1, 0.0, 0.5), 96, 64, sun=sun, flags=fl)
            img, st = sc.render(fr, stats=True)
            ref, ost = o.render(fr.params, 96, 64)
            d = (img.view(np.uint32) != ref.view(np.uint32)).any(axis=2)
            print(el, az, fl, "pixels differing", int(d.sum()), "fetches", st.as_dict()["shadow_fetches"],
                  ost.as_dict()["shadow_fetches"], flush=True)
            if d.any():
                ys, xs = np.nonzero(d)
                for y, x in list(zip(ys, xs))[:3]:
                    print("   px", x, y, img[y, x], ref[y, x], flush=True)
    sc.close()


if __name__ == "__main__":
    main()
