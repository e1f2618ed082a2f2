"""Host-side cost of one frame submission (Python -> ctypes -> vx_render ->
hipLaunchKernelGGL) against the kernel time: if submitting takes longer than
the kernel runs, the GPU idles between frames and the bench is host-bound.
usage: python tools/enqueue_rate.py [--config C3] [--flags 48] [--frames 400]"""
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
    up = 3.0 if cfg["scene"] == "s_up3" else 1.0
    sc = vx.Scene(map_bytes=grid.tobytes(), map_format=vx.FORMAT_GRID, dims=(X, Y, Z), device=0)
    fr = presets.camera_frame(cfg["camera"], cfg["w"], cfg["h"], scale=up, flags=a.flags)
    out = torch.empty(cfg["w"] * cfg["h"] * 4, dtype=torch.uint8, device="cuda")
    st = torch.cuda.Stream()
    torch.cuda.set_stream(st)
    for _ in range(200):
        sc.render_device(fr, out.data_ptr(), pixel_format=vx.PIXEL_RGBA8, stream=st.cuda_stream)
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    t0 = time.perf_counter()
    e0.record()
    for _ in range(a.frames):
        sc.render_device(fr, out.data_ptr(), pixel_format=vx.PIXEL_RGBA8, stream=st.cuda_stream)
    t_sub = time.perf_counter() - t0
    e1.record()
    torch.cuda.synchronize()
    t_all = time.perf_counter() - t0
    print(f"{a.config} flags={a.flags}: submit {1e3 * t_sub / a.frames:.4f} ms/frame (host), "
          f"events {e0.elapsed_time(e1) / a.frames:.4f} ms/frame, wall {1e3 * t_all / a.frames:.4f} ms/frame")
    sc.close()


if __name__ == "__main__":
    main()
