"""How much of a frame is kernel tail?  Frames on one stream vs alternating
between two streams (two framebuffers, double buffering): with two streams the
next frame's waves fill the CUs the previous frame's last waves leave idle.
usage: python tools/overlap_probe.py [--flags 48] [--frames 400]"""
import argparse
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="C3")
    ap.add_argument("--flags", type=int, default=48)
    ap.add_argument("--frames", type=int, default=400)
    a = ap.parse_args()
    import torch
    import voxmap_amd as vx
    from voxmap_amd import presets
    cfg = presets.CONFIGS[a.config]
    grid = presets.scene_grid(cfg["scene"])
    Z, Y, X = grid.shape
    sc = vx.Scene(map_bytes=grid.tobytes(), map_format=vx.FORMAT_GRID, dims=(X, Y, Z), device=0)
    fr = presets.camera_frame(cfg["camera"], cfg["w"], cfg["h"], flags=a.flags)
    n = cfg["w"] * cfg["h"] * 4
    outs = [torch.empty(n, dtype=torch.uint8, device="cuda") for _ in range(2)]
    streams = [torch.cuda.Stream(), torch.cuda.Stream()]

    def run(k_streams, frames):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for i in range(frames):
            j = i % k_streams
            sc.render_device(fr, outs[j].data_ptr(), pixel_format=vx.PIXEL_RGBA8, stream=streams[j].cuda_stream)
        torch.cuda.synchronize()
        return 1e3 * (time.perf_counter() - t0) / frames

    run(1, 1500)                     # clock settle
    res = {1: [], 2: []}
    for _ in range(5):
        for k in (1, 2):
            res[k].append(run(k, a.frames))
    for k in (1, 2):
        print(f"{a.config} flags={a.flags} streams={k}: {min(res[k]):.4f} ms/frame (min of 5), "
              f"median {sorted(res[k])[2]:.4f}")
    sc.close()


if __name__ == "__main__":
    main()
