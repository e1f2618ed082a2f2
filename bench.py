#!/usr/bin/env python3
"""Benchmark of the Voxmap shading path on MI355X (BASELINE.json metric).

A step renders one full frame of the headline workload (BASELINE configs[2],
C3: 3840x2160 "full quality" = the reference's v1 shading (primary visibility +
sun march + AO + sky/clouds + glass) + the f-3 extensions reflection and rough
normals, on the synthetic S-proc 1024x256x32 field, camera K1) from the
HBM-resident field into an HBM-resident RGBA8 framebuffer.  The v1 shading
alone (the reference's own shader, flags 0) is timed in the same run and
reported under config.v1.  --config C5: the 3^3-upscaled 3072x768x96 field
with 16-sample soft shadows (BASELINE configs[4]).

N > 1 GPUs (one process per GPU, torchrun): weak scaling — the frame grows
with N (W = 3840*sqrt(N), H = 2160*sqrt(N), so N = 4 is C4's 7680x4320),
64x64 screen tiles are dealt round-robin to ranks, each rank renders its tiles
and rank 0 gathers them over RCCL (torch.distributed "nccl") and de-tiles; the
gather is inside the timed step.

Prints ONE JSON line on rank 0.
"""
from __future__ import annotations

import argparse
import json
import math
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

HBM_PEAK_GBPS = 8000.0  # MI355X HBM3E spec peak (MI355X_MICROARCH.md chip table)
TILE = 64


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=100)
    ap.add_argument("--warmup", type=int, default=10)
    ap.add_argument("--inflight", type=int, default=2,
                    help="frames in flight: consecutive frames alternate over this many streams and framebuffers "
                         "(double buffering), so one frame's launch gap and tail overlap the next (~6%%, "
                         "profiles/r01_overlap.txt); 1 = one stream")
    ap.add_argument("--settle-ms", type=float, default=300.0,
                    help="untimed frames rendered before the warmup so the GPU clock leaves its idle state "
                         "(a ~5 ms burst runs ~12%% slower than steady state: profiles/r01_clock_settle.txt)")
    ap.add_argument("--config", default="C3")
    ap.add_argument("--camera", default=None)
    ap.add_argument("--cpu-seconds", type=float, default=12.0, help="target CPU-baseline sample time")
    ap.add_argument("--no-cpu", action="store_true")
    ap.add_argument("--quality", choices=["full", "v1"], default="full",
                    help="full = v1 + REFLECT + ROUGH (BASELINE 'full quality'); v1 = the reference shader only")
    ap.add_argument("--flags", type=int, default=None, help="VX_FLAG_* bits overriding --quality (diagnostics)")
    ap.add_argument("--samples", type=int, default=None, help="soft-shadow samples (default: 16 for C5, else 1)")
    ap.add_argument("--sun-radius", type=float, default=0.03)
    ap.add_argument("--traffic-json", default=None,
                    help="per-launch HBM bytes measured by rocprofv3 PMC (tools/pmc_traffic.py)")
    return ap.parse_args()


def main():
    args = parse()
    import numpy as np
    import torch
    import torch.distributed as dist

    import voxmap_amd as vx
    from voxmap_amd import presets

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus:
        if args.gpus > 1 and world == 1:
            raise SystemExit("--gpus N>1 must be launched with torch.distributed.run (one process per GPU)")
        world = max(world, 1)
    torch.cuda.set_device(local)
    if world > 1:
        dist.init_process_group("nccl", device_id=torch.device("cuda", local))

    cfg = presets.CONFIGS[args.config]
    cam = args.camera or cfg["camera"]
    scale = math.sqrt(world)
    W = int(round(cfg["w"] * scale / 16)) * 16
    H = int(round(cfg["h"] * scale / 16)) * 16
    up = 3.0 if cfg["scene"] == "s_up3" else 1.0

    grid = presets.scene_grid(cfg["scene"])
    Z, Y, X = grid.shape
    noise = vx.noise_synth(0)
    t_scene = time.perf_counter()
    # palette grid in, distance field + octant copies built on the device (f-1)
    scene = vx.Scene(map_bytes=grid.tobytes(), map_format=vx.FORMAT_GRID, noise_bytes=noise.tobytes(),
                     noise_format=vx.FORMAT_BIN, dims=(X, Y, Z), device=local)
    t_scene = time.perf_counter() - t_scene
    flags = args.flags if args.flags is not None else (vx.FLAG_FULL_QUALITY if args.quality == "full" else 0)
    samples = args.samples if args.samples is not None else cfg.get("samples", 1)
    frame = presets.camera_frame(cam, W, H, scale=up, flags=flags, shadow_samples=samples,
                                 sun_radius=args.sun_radius if samples > 1 else 0.0)
    # K frames in flight: frame i renders on stream i % K into framebuffer
    # i % K (a swap chain); real streams, so torch events and kernels share them
    K = max(1, args.inflight)
    streams = [torch.cuda.Stream() for _ in range(K)]
    torch.cuda.set_stream(streams[0])
    stream = streams[0].cuda_stream

    tiles_x, tiles_y = -(-W // TILE), -(-H // TILE)
    n_tiles = tiles_x * tiles_y
    if world == 1:
        outs = [torch.empty(H * W * 4, dtype=torch.uint8, device="cuda") for _ in range(K)]
        out = outs[0]

        def make_step(j):
            o, sj = outs[j], streams[j].cuda_stream
            return lambda: scene.render_device(frame, o.data_ptr(), pixel_format=vx.PIXEL_RGBA8, stream=sj)

        st = scene.render_device(frame, out.data_ptr(), pixel_format=vx.PIXEL_RGBA8, stream=stream, stats=True)
        stats = st.as_dict()
    else:
        from voxmap_amd.dist import ShardedFrame, TileLayout
        layout = TileLayout(W, H, TILE)
        shards = []
        for j in range(K):
            sj = streams[j].cuda_stream
            shards.append(ShardedFrame(
                dist, layout, 4, torch.uint8, "cuda",
                render_tiles=lambda ids, buf, sj=sj: scene.render_tiles(frame, TILE, ids, buf.data_ptr(),
                                                                        pixel_format=vx.PIXEL_RGBA8, stream=sj),
                detile=lambda ids, cat, fr, sj=sj: scene.detile(W, H, TILE, ids, cat.data_ptr(), fr.data_ptr(),
                                                                pixel_format=vx.PIXEL_RGBA8, stream=sj)))

        def make_step(j):
            sh, strm = shards[j], streams[j]

            def f():
                with torch.cuda.stream(strm):      # the gather and de-tile follow this frame's stream
                    sh.step()
            return f

        sharded = shards[0]
        st = scene.render_tiles(frame, TILE, layout.rank_tiles(world, rank), sharded.buf.data_ptr(),
                                pixel_format=vx.PIXEL_RGBA8, stream=stream, stats=True)
        keys = [k for k in st.as_dict().keys() if k != "kernel_ms"]
        vec = torch.tensor([float(st.as_dict()[k]) for k in keys], dtype=torch.float64, device="cuda")
        dist.all_reduce(vec)
        stats = {k: float(v) for k, v in zip(keys, vec.tolist())}
        stats["kernel_ms"] = float(st.kernel_ms)
    step_fns = [make_step(j) for j in range(K)]
    n_done = [0]

    def step():
        step_fns[n_done[0] % K]()
        n_done[0] += 1

    # clock settle: every rank renders the same number of untimed frames (the
    # sharded step holds a collective), sized from a short probe to ~settle_ms
    settle_steps = 0
    if args.settle_ms > 0:
        torch.cuda.synchronize()
        tp = time.perf_counter()
        for _ in range(3):
            step()
        torch.cuda.synchronize()
        probe_ms = 1000.0 * (time.perf_counter() - tp) / 3
        n = torch.tensor([math.ceil(args.settle_ms / max(probe_ms, 1e-3))], dtype=torch.int64,
                         device="cuda" if world > 1 else "cpu")
        if world > 1:
            dist.all_reduce(n, op=dist.ReduceOp.MAX)
        settle_steps = int(min(int(n.item()), 20000)) + 3
        for _ in range(settle_steps - 3):
            step()
    for _ in range(args.warmup):
        step()
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        step()
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    wall = time.perf_counter() - t0
    ev_ms = None
    if world == 1:
        # per-launch kernel time for the roofline: the same frames on ONE stream,
        # HIP events on that stream (no overlap; agrees with rocprofv3's average)
        one = make_step(0)
        ev0 = torch.cuda.Event(enable_timing=True)
        ev1 = torch.cuda.Event(enable_timing=True)
        torch.cuda.synchronize()
        ev0.record()
        for _ in range(args.steps):
            one()
        ev1.record()
        torch.cuda.synchronize()
        ev_ms = ev0.elapsed_time(ev1) / args.steps
    t_local = wall
    if world > 1:
        tt = torch.tensor([wall], dtype=torch.float64, device="cuda")
        dist.all_reduce(tt, op=dist.ReduceOp.MAX)
        t_local = float(tt.item())
    ms_per_step = 1000.0 * t_local / args.steps

    v1 = None
    if world == 1 and flags != 0 and args.flags is None and samples <= 1:
        # the reference's own shader (v1, flags 0) on the same frame: the same
        # K-in-flight wall timing, and one stream with events for its roofline
        fr1 = presets.camera_frame(cam, W, H, scale=up)
        st1 = scene.render_device(fr1, out.data_ptr(), pixel_format=vx.PIXEL_RGBA8, stream=stream, stats=True)
        v1fns = [(lambda o=outs[j], sj=streams[j].cuda_stream:
                  scene.render_device(fr1, o.data_ptr(), pixel_format=vx.PIXEL_RGBA8, stream=sj)) for j in range(K)]
        for i in range(args.warmup):
            v1fns[i % K]()
        torch.cuda.synchronize()
        tw = time.perf_counter()
        for i in range(args.steps):
            v1fns[i % K]()
        torch.cuda.synchronize()
        ms1w = 1000.0 * (time.perf_counter() - tw) / args.steps
        e0 = torch.cuda.Event(enable_timing=True)
        e1 = torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(args.steps):
            v1fns[0]()
        e1.record()
        torch.cuda.synchronize()
        ms1 = e0.elapsed_time(e1) / args.steps
        r1 = st1.pixels + st1.shadow_rays
        v1 = {"ms_per_frame": round(ms1w, 4), "mrays_per_s": round(r1 / ms1w / 1e3, 3), "rays_per_frame": int(r1),
              "single_stream_ms_per_frame": round(ms1, 4), "alg_bytes": int(st1.alg_bytes),
              "roofline_frac": round(st1.alg_bytes / (ms1 * 1e-3) / 1e9 / HBM_PEAK_GBPS, 4)}

    rays = stats["pixels"] + stats["shadow_rays"] + stats["reflect_rays"]   # rays actually marched per frame
    value = rays * args.steps / t_local / 1e6                 # whole-job Mrays/s
    result = None
    if rank == 0:
        per_launch_bytes = float(stats["alg_bytes"]) / world if world > 1 else float(stats["alg_bytes"])
        kernel_ms = ev_ms if world == 1 else stats["kernel_ms"]
        achieved = per_launch_bytes / (kernel_ms * 1e-3) / 1e9
        traffic = None
        tj_path = args.traffic_json or os.path.join(
            ROOT, "profiles", "traffic_r01.json" if args.config != "C5" else "traffic_r01_c5.json")
        if world == 1 and os.path.exists(tj_path):
            try:
                tj = json.load(open(tj_path))
                if (tj.get("config") == args.config and tj.get("camera") == cam and tj.get("flags", 0) == flags
                        and tj.get("samples", 1) == samples):
                    traffic = tj.get("hbm_bytes_per_launch")
            except Exception:
                traffic = None
        result = {
            "metric": f"Mrays/s at {cfg['w']}x{cfg['h']} {'full quality' if flags else 'v1 shading'} "
                      f"({args.config}); fps; % HBM roofline",
            "value": round(value, 3),
            "unit": "Mrays/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(ms_per_step, 4),
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "fp32",
            "data": f"synthetic {cfg['scene']} field (seed 1) in map.bin layout; synthetic noise texture (real "
                    "map.blob is AES-encrypted, key not in repo)",
            "config": {
                "workload": f"{args.config}: {W}x{H} frame, " + (
                    "full quality = v1 shading (primary visibility + sun march + trilinear AO + sky/clouds + glass) "
                    "+ ext reflection + rough normals" if flags == vx.FLAG_FULL_QUALITY else
                    f"v1 shading flags={flags}") +
                    (f" + {samples}-sample soft shadows (sun radius {args.sun_radius})" if samples > 1 else "") +
                    f", field {X}x{Y}x{Z}, camera {cam}, sun hour 1.0, RGBA8 framebuffer in HBM",
                "flags": flags, "shadow_samples": samples, "scene_build_s": round(t_scene, 3),
                "clock_settle": {"ms": args.settle_ms, "untimed_frames": settle_steps},
                "width": W, "height": H, "field": [X, Y, Z], "camera": cam,
                "tiles": {"size": TILE, "count": n_tiles, "assignment": "round-robin"} if world > 1 else None,
                "fps": round(1000.0 / ms_per_step, 2),
                "inflight": {"frames": K, "streams": K, "framebuffers": K,
                             "single_stream_ms_per_frame": round(ev_ms, 4) if ev_ms is not None else None},
                "rays_per_frame": int(rays), "primary_rays": int(stats["pixels"]),
                "shadow_rays": int(stats["shadow_rays"]), "reflect_rays": int(stats["reflect_rays"]),
                "mrays_per_s_nominal_2rpp": round(2 * stats["pixels"] * args.steps / t_local / 1e6, 3),
                "v1": v1,
            },
            "roofline": {
                "bound": "hbm",
                "kernel": "k_render (fused primary visibility + shading + sun march" +
                          (" + reflection walk" if flags & vx.FLAG_REFLECT else "") + ")",
                "achieved": round(achieved, 2),
                "peak": HBM_PEAK_GBPS,
                "unit": "GB/s",
                "frac": round(achieved / HBM_PEAK_GBPS, 4),
                "traffic": traffic,
                "alg_bytes_per_launch": int(per_launch_bytes),
                "avg_launch_ms": round(kernel_ms, 4),
            },
        }
        if world == 1 and not args.no_cpu:
            result["cpu_baseline"] = cpu_baseline(scene, noise, frame, W, H, args.cpu_seconds)
    scene.close()
    if world > 1:
        dist.barrier()
        dist.destroy_process_group()
    if rank == 0:
        print(json.dumps(result), flush=True)


def cpu_baseline(scene, noise, frame, W, H, target_s):
    """The scalar oracle (oracle/, -O2 -fno-fast-math -ffp-contract=off, OpenMP
    over rows) on a bounded sample of the same frame: whole frames repeated
    until ~target_s when a frame is cheap (median rate reported), else a
    deterministic 1-in-k row subset sized to ~target_s."""
    import numpy as np

    import oracle
    threads = int(os.environ.get("OMP_NUM_THREADS", "0")) or min(16, os.cpu_count() or 1)
    threads = max(1, min(threads, 16))
    dev_field = scene.read_field()            # same bytes (A channel included) the GPU marched
    o = oracle.Oracle(dev_field, noise)
    out = np.empty((H, W, 4), np.float32)
    k = 64
    t0 = time.perf_counter()
    _, st = o.render(frame.params, W, H, row0=k // 2, row_step=k, threads=threads, out=out)
    est_full = (time.perf_counter() - t0) * k
    rates, desc = [], ""
    if est_full * 3 <= target_s:
        reps = max(3, int(target_s / max(est_full, 1e-3)))
        for _ in range(reps):
            t0 = time.perf_counter()
            _, st = o.render(frame.params, W, H, threads=threads, out=out)
            dt = time.perf_counter() - t0
            rates.append((st.pixels + st.shadow_rays + st.reflect_rays) / dt / 1e6)
        desc = (f"{reps} full {W}x{H} frames ({st.pixels} pixels, {st.pixels + st.shadow_rays + st.reflect_rays} "
                f"rays each), median rate")
    else:
        k = max(1, int(math.ceil(est_full / target_s)))
        t0 = time.perf_counter()
        _, st = o.render(frame.params, W, H, row0=k // 2, row_step=k, threads=threads, out=out)
        dt = time.perf_counter() - t0
        rates.append((st.pixels + st.shadow_rays + st.reflect_rays) / dt / 1e6)
        desc = f"rows {k // 2}::{k} of the same {W}x{H} frame ({st.pixels} pixels) in {dt:.2f} s"
    return {
        "value": round(float(np.median(rates)), 4),
        "unit": "Mrays/s",
        "cores": threads,
        "kind": "port",
        "sample": desc,
    }


if __name__ == "__main__":
    main()
