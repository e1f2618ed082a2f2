"""GPU check of the tile entry box: frames rendered without stats (the path
that runs k_tile_box) against the oracle, word for word, at the BASELINE
sizes and on small scenes.  usage: python tools/tile_box_check.py"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    import numpy as np
    import oracle
    import voxmap_amd as vx
    from voxmap_amd import presets, scenes
    noise = scenes.real_noise()
    bad_total = 0
    field = vx.field_build(presets.scene_grid("s_proc"))
    O = oracle.Oracle(field, noise, exit=True)
    with vx.Scene(map_bytes=field.tobytes(), map_format=vx.FORMAT_BIN, noise_bytes=noise.tobytes(),
                  noise_format=vx.FORMAT_BIN, dims=(1024, 256, 32), device=0) as sc:
        for cam, w, h, fl in (("K1", 3840, 2160, 48), ("K1", 3840, 2160, 0), ("K0", 1920, 1080, 0),
                              ("K2", 1920, 1080, 0), ("K1", 333, 201, 48)):
            fr = presets.camera_frame(cam, w, h, flags=fl)
            img, _ = sc.render(fr)
            ref, _ = O.render(fr.params, w, h, threads=16)
            bad = int(np.count_nonzero(np.any(img.view(np.uint32) != ref.view(np.uint32), axis=2)))
            bad_total += bad
            print(cam, w, h, fl, "pixels differing", bad, flush=True)
    for seed, dims in ((5, (96, 48, 16)), (11, (128, 64, 24))):
        field = vx.field_build(scenes.small_proc(seed, dims=dims, n_boxes=16, n_glass=6))
        O = oracle.Oracle(field, noise, exit=True)
        with vx.Scene(map_bytes=field.tobytes(), map_format=vx.FORMAT_BIN, noise_bytes=noise.tobytes(),
                      noise_format=vx.FORMAT_BIN, dims=dims, device=0) as sc:
            for rot in ((1.1, 0.0, 0.6), (1.45, 0.0, -1.57), (1.3, 0.0, 2.4)):
                fr = vx.make_frame((dims[0] / 2, dims[1] / 2, 18.0), rot, 320, 200, flags=48)
                img, _ = sc.render(fr)
                ref, _ = O.render(fr.params, 320, 200)
                bad = int(np.count_nonzero(np.any(img.view(np.uint32) != ref.view(np.uint32), axis=2)))
                bad_total += bad
                print("small", seed, rot, "pixels differing", bad, flush=True)
    print("total differing pixels", bad_total)
    sys.exit(1 if bad_total else 0)


if __name__ == "__main__":
    main()
