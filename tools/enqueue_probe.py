"""Host enqueue cost of vx_render against the frame time (is a stream of
frames host-bound?): per flags, the host time to enqueue N frames on two
streams without waiting, then the wall time until they finish.
usage: python tools/enqueue_probe.py [--config C3] [--flags 0,48]"""
import argparse
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="C3")
    ap.add_argument("--flags", default="0,48")
    ap.add_argument("--frames", type=int, default=400)
    args = ap.parse_args()
    import torch

    import voxmap_amd as vx
    from voxmap_amd import presets, scenes
    cfg = presets.CONFIGS[args.config]
    grid = presets.scene_grid(cfg["scene"])
    Z, Y, X = grid.shape
    W, H = cfg["w"], cfg["h"]
    sc = vx.Scene(map_bytes=grid.tobytes(), map_format=vx.FORMAT_GRID, noise_path=scenes.NOISE_PATH,
                  dims=(X, Y, Z), device=0)
    streams = [torch.cuda.Stream(), torch.cuda.Stream()]
    outs = [torch.empty(W * H * 4, dtype=torch.uint8, device="cuda") for _ in range(2)]
    for flags in [int(f) for f in args.flags.split(",")]:
        fr = presets.camera_frame(cfg["camera"], W, H, flags=flags)
        for _ in range(300):
            sc.render_device(fr, outs[0].data_ptr(), pixel_format=vx.PIXEL_RGBA8, stream=streams[0].cuda_stream)
        torch.cuda.synchronize()
        for ns in (1, 2):
            t0 = time.perf_counter()
            for i in range(args.frames):
                j = i % ns
                sc.render_device(fr, outs[j].data_ptr(), pixel_format=vx.PIXEL_RGBA8, stream=streams[j].cuda_stream)
            t1 = time.perf_counter()
            torch.cuda.synchronize()
            t2 = time.perf_counter()
            print(f"flags={flags:3d} streams={ns}: host enqueue {1e6 * (t1 - t0) / args.frames:7.1f} us/frame, "
                  f"wall {1e6 * (t2 - t0) / args.frames:7.1f} us/frame", flush=True)
    sc.close()


if __name__ == "__main__":
    main()
