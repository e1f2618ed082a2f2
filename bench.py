#!/usr/bin/env python3
"""Benchmark of the Voxmap shading path on MI355X (BASELINE.json metric).

A step renders one full frame of the headline workload (BASELINE configs[2],
C3: 3840x2160 "full quality" = the reference's v1 shading (primary visibility +
sun march + AO + sky/clouds + glass) + the f-3 extensions reflection and rough
normals, on the synthetic S-proc 1024x256x32 field, camera K1, the reference's
own res/noise.bin.gz) from the HBM-resident field into an HBM-resident RGBA8
framebuffer.  In the same N = 1 run: the v1 shading alone (config.v1),
BASELINE configs[4] C5 (3^3-upscaled 3072x768x96 field, 16-sample soft
shadows; config.c5) and the frame rate with the framebuffer copied to pinned
host memory (config.fps_with_d2h, SURVEY §8d: kernel + D2H).  --config C5
makes C5 the headline.

N > 1 GPUs, one process per GPU: launched by torch.distributed.run, or by
``python bench.py --gpus N`` itself, which starts N rank processes (fresh
interpreters, before anything touches a GPU) and exits with their status.  The
frame is cut into 64-row full-width bands dealt round-robin; each rank renders
its bands in place and rank 0 gathers them into its frame over RCCL
(vx_mgpu_render: native C++, ncclSend/ncclRecv in one group; --gather torch
runs the same protocol through torch.distributed).  The gather is inside the
timed step.  The default config for N > 1 is BASELINE configs[3], C4:
7680x4320 for every N (strong scaling); --config C3 grows the frame with N
instead (3840*sqrt(N) x 2160*sqrt(N), weak scaling).

--standin (tests only): the same orchestration (rank spawn, barriers, band
deal, gather, max-over-ranks timing, the JSON line) on CPU over gloo, with a
stand-in band renderer instead of the HIP library -- what
tests/test_bench_spawn.py runs.

Prints ONE JSON line on rank 0.
"""
from __future__ import annotations

import argparse
import json
import math
import os
import socket
import subprocess
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

HBM_PEAK_GBPS = 8000.0  # MI355X HBM3E spec peak (MI355X_MICROARCH.md chip table)
PMC_TAG = "r06"         # profiles/{traffic,valu}_<tag>[_c5].json: this round's rocprofv3 PMC summaries


def parse(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=100)
    ap.add_argument("--warmup", type=int, default=10)
    ap.add_argument("--inflight", type=int, default=None,
                    help="frames in flight: consecutive frames alternate over this many streams and framebuffers "
                         "(a swap chain), so one frame's ramp-down overlaps the next frames' blocks. Default 4 on "
                         "one GPU (one stream per hardware queue: C3 full quality -4.8 %% against 2, "
                         "profiles/r03_ab_row_stride.txt), 2 at N > 1 (the RCCL gathers share one communicator); "
                         "1 = one stream")
    ap.add_argument("--settle-ms", type=float, default=300.0,
                    help="untimed frames rendered before the warmup so the GPU clock leaves its idle state "
                         "(a ~5 ms burst runs ~12%% slower than steady state: profiles/r01_clock_settle.txt)")
    ap.add_argument("--config", default=None, choices=["C2", "C3", "C4", "C5"],
                    help="default: C3 on one GPU, C4 (7680x4320, BASELINE configs[3]) on N > 1")
    ap.add_argument("--camera", default=None)
    ap.add_argument("--cpu-seconds", type=float, default=12.0, help="target CPU-baseline sample time")
    ap.add_argument("--no-cpu", action="store_true")
    ap.add_argument("--no-c5", action="store_true", help="skip the secondary C5 measurement of an N = 1 C3 run")
    ap.add_argument("--no-d2h", action="store_true", help="skip the kernel + D2H frame rate of an N = 1 run")
    ap.add_argument("--quality", choices=["full", "v1"], default="full",
                    help="full = v1 + REFLECT + ROUGH (BASELINE 'full quality'); v1 = the reference shader only")
    ap.add_argument("--flags", type=int, default=None, help="VX_FLAG_* bits overriding --quality (diagnostics)")
    ap.add_argument("--samples", type=int, default=None, help="soft-shadow samples (default: 16 for C5, else 1)")
    ap.add_argument("--sun-radius", type=float, default=0.03)
    ap.add_argument("--gather", choices=["native", "torch", "gloo"], default="native",
                    help="N > 1: native = vx_mgpu_render (RCCL from C++); torch = the same bands over "
                         "torch.distributed 'nccl'; gloo = a rehearsal on ONE GPU (RCCL refuses two ranks on "
                         "one device): every rank renders its bands on the GPU (VOXMAP_BENCH_DEVICE, default "
                         "LOCAL_RANK), the bands travel over gloo through host memory, and rank 0 checks the "
                         "gathered frame against a whole-frame vx_render (config.gather_frame_ok); not a timing")
    ap.add_argument("--standin", action="store_true", help=argparse.SUPPRESS)
    return ap.parse_args(argv)


# ---------------------------------------------------------------- rank spawn
def _free_port() -> int:
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def spawn_ranks(n: int, argv) -> int:
    """``bench.py --gpus N`` without a launcher: start N rank processes of this
    script (fresh interpreters: nothing in this process has touched a GPU, and
    nothing is exec'd), the torch.distributed.run environment set for each,
    and return the first non-zero exit status.  Rank 0 prints the JSON line."""
    port = _free_port()
    procs = []
    for r in range(n):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(n), LOCAL_WORLD_SIZE=str(n),
                   GROUP_RANK="0", MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port),
                   HSA_ENABLE_IPC_MODE_LEGACY=os.environ.get("HSA_ENABLE_IPC_MODE_LEGACY", "0"))
        procs.append(subprocess.Popen([sys.executable, os.path.abspath(__file__), *argv], env=env))
    rc = 0
    try:
        for p in procs:
            code = p.wait()
            if code and not rc:
                rc = code
                for q in procs:                 # one rank failed: the others would wait at a barrier forever
                    if q.poll() is None:
                        q.terminate()
    finally:
        for p in procs:
            if p.poll() is None:
                p.kill()
                p.wait()
    return rc


# ---------------------------------------------------------------- timing
REPEATS = 7             # timed blocks of `steps` frames each; the line reports their median


def timed(sync, step, steps, warmup, settle_ms, dist=None, sync_dev=None, repeats=1):
    """Settle the clock, warm up, then time `repeats` blocks of exactly `steps`
    frames, each bracketed by a barrier and a device synchronise on both sides
    (max over ranks taken by the caller).  Returns the blocks' wall times (s)."""
    import torch
    settle = 0
    if settle_ms > 0:
        sync()
        tp = time.perf_counter()
        for _ in range(3):
            step()
        sync()
        probe_ms = 1000.0 * (time.perf_counter() - tp) / 3
        n = torch.tensor([math.ceil(settle_ms / max(probe_ms, 1e-3))], dtype=torch.int64)
        if dist is not None:
            if sync_dev is not None:
                n = n.to(sync_dev)
            dist.all_reduce(n, op=dist.ReduceOp.MAX)     # equal frame counts: the step is collective
        settle = int(min(int(n.item()), 20000)) + 3
        for _ in range(settle - 3):
            step()
    for _ in range(warmup):
        step()
    walls = []
    for _ in range(max(1, repeats)):
        sync()
        if dist is not None:
            dist.barrier()
        sync()
        t0 = time.perf_counter()
        for _ in range(steps):
            step()
        sync()
        if dist is not None:
            dist.barrier()
        sync()
        walls.append(time.perf_counter() - t0)
    return walls, settle


def block_summary(walls, steps):
    """Median block time and the spread of the timed blocks (the line's ms_per_step is the median)."""
    ms = sorted(1000.0 * w / steps for w in walls)
    med = ms[len(ms) // 2] if len(ms) % 2 else 0.5 * (ms[len(ms) // 2 - 1] + ms[len(ms) // 2])
    return med, {"blocks": len(ms), "steps_per_block": steps, "ms_per_step_blocks": [round(v, 4) for v in ms],
                 "median_ms_per_step": round(med, 4), "spread_pct": round(100.0 * (ms[-1] - ms[0]) / med, 2),
                 "how": "each block: exactly `steps` frames between a barrier + device synchronise on both sides; "
                        "value and ms_per_step from the median block"}


def event_ms(torch, one, steps):
    """Average per-frame kernel time of `one` on the CURRENT stream (the one it
    launches on), HIP events on that stream, no overlap between frames."""
    ev0 = torch.cuda.Event(enable_timing=True)
    ev1 = torch.cuda.Event(enable_timing=True)
    torch.cuda.synchronize()
    ev0.record()
    for _ in range(steps):
        one()
    ev1.record()
    torch.cuda.synchronize()
    return ev0.elapsed_time(ev1) / steps


def pmc_entry(name, config, cam, flags, samples):
    """A committed rocprofv3 PMC summary (tools/prof_summary.py) for this workload, if any."""
    path = os.path.join(ROOT, "profiles", name)
    if not os.path.exists(path):
        return None
    try:
        tj = json.load(open(path))
    except Exception:
        return None
    if (tj.get("config") == config and tj.get("camera") == cam and tj.get("flags", 0) == flags
            and tj.get("samples", 1) == samples):
        return tj
    return None


def exit_tables(torch, vx, scene, frame, W, H):
    """The sun exit copy this frame's march reads (DESIGN.md §3 "Sun exit
    tables"): which one, the time to build it (vx_prepare_sun on a scene that
    has not built it yet: a cone copy is built once per sun octant and window,
    and the sun moves ~1 rad per hour, map.js:399), and the shadow fetches of
    the same frame without tables -- the reference's own step count."""
    st = torch.cuda.Stream()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    info = scene.prepare_sun(frame, stream=st.cuda_stream)
    info["build_ms"] = round(info["build_ms"], 4)                 # GPU time (HIP events) of the build
    info["prepare_wall_ms"] = round(1000.0 * (time.perf_counter() - t0), 3)   # + first allocation, host
    fl = vx.Frame(frame.params.copy(), W, H)
    fl.params.flags |= vx.FLAG_NO_EXIT
    out = torch.empty(H * W * 4, dtype=torch.uint8, device="cuda")
    s0 = scene.render_device(fl, out.data_ptr(), pixel_format=vx.PIXEL_RGBA8, stream=st.cuda_stream,
                             stats=True).as_dict()
    info["reference_shadow_fetches"] = int(s0["shadow_fetches"])
    info["reference_alg_bytes"] = int(s0["alg_bytes"])
    info["kinds"] = "0 none, 1 orthant copies (any sun of the octant), 2 cone copy {octant, kx, ky}"
    return info


def single_gpu(torch, vx, scene, frame, W, H, K, steps, warmup, settle_ms, repeats=REPEATS):
    """N = 1: K frames in flight over K streams/framebuffers; timings + stats."""
    ex = exit_tables(torch, vx, scene, frame, W, H)
    streams = [torch.cuda.Stream() for _ in range(K)]
    torch.cuda.set_stream(streams[0])
    outs = [torch.empty(H * W * 4, dtype=torch.uint8, device="cuda") for _ in range(K)]
    fns = [(lambda o=outs[j], sj=streams[j].cuda_stream:
            scene.render_device(frame, o.data_ptr(), pixel_format=vx.PIXEL_RGBA8, stream=sj)) for j in range(K)]
    st = scene.render_device(frame, outs[0].data_ptr(), pixel_format=vx.PIXEL_RGBA8,
                             stream=streams[0].cuda_stream, stats=True)
    n = [0]

    def step():
        fns[n[0] % K]()
        n[0] += 1
    walls, settle = timed(torch.cuda.synchronize, step, steps, warmup, settle_ms, repeats=repeats)
    med, blocks = block_summary(walls, steps)
    ev = sorted(event_ms(torch, fns[0], steps) for _ in range(3))[1]
    return {"wall_s": med * steps / 1000.0, "blocks": blocks, "settle": settle, "ev_ms": ev, "stats": st.as_dict(),
            "exit": ex}


def fps_with_d2h(torch, vx, scene, frame, W, H, frames, K=2):
    """SURVEY §8d's fps: kernel + the RGBA8 framebuffer copied to pinned host
    memory.  K framebuffers; frame i renders into fb[i % K] on the render stream
    and is copied out on a second stream while frame i + 1 renders (the render
    into fb[j] waits for that buffer's previous copy)."""
    rs, cs = torch.cuda.Stream(), torch.cuda.Stream()
    fbs = [torch.empty(H * W * 4, dtype=torch.uint8, device="cuda") for _ in range(K)]
    hosts = [torch.empty(H * W * 4, dtype=torch.uint8, pin_memory=True) for _ in range(K)]
    copied = [None] * K

    def one(i):
        j = i % K
        if copied[j] is not None:
            rs.wait_event(copied[j])
        scene.render_device(frame, fbs[j].data_ptr(), pixel_format=vx.PIXEL_RGBA8, stream=rs.cuda_stream)
        done = torch.cuda.Event()
        done.record(rs)
        cs.wait_event(done)
        with torch.cuda.stream(cs):
            hosts[j].copy_(fbs[j], non_blocking=True)
        copied[j] = torch.cuda.Event()
        copied[j].record(cs)
    for i in range(4):
        one(i)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for i in range(frames):
        one(i)
    torch.cuda.synchronize()
    ms = 1000.0 * (time.perf_counter() - t0) / frames
    # the copy alone (one stream, same bytes) to show what binds
    torch.cuda.synchronize()
    t1 = time.perf_counter()
    for i in range(frames):
        hosts[i % K].copy_(fbs[i % K], non_blocking=True)
    torch.cuda.synchronize()
    copy_ms = 1000.0 * (time.perf_counter() - t1) / frames
    return {"fps": round(1000.0 / ms, 2), "ms_per_frame": round(ms, 4), "frames": frames,
            "d2h_bytes_per_frame": H * W * 4, "d2h_alone_ms": round(copy_ms, 4),
            "d2h_gbps": round(H * W * 4 / (copy_ms * 1e-3) / 1e9, 2),
            "how": f"{K} framebuffers; render on one stream, RGBA8 copy to pinned host memory on a second, "
                   "overlapped with the next frame's render"}


def bound_of(pmc):
    """The unit that measurably binds the kernel, from the committed PMC summary:
    VALU issue (valu_busy is a lower bound: 2 cycles per instruction) or the CU's
    texture address / data path (TA / TD busy, one per CU for its 4 SIMDs); the
    field is cache-resident, so HBM is never it (roofline.traffic << algorithmic)."""
    if not pmc:
        return "hbm"
    td = max(pmc.get("ta_busy") or 0.0, pmc.get("td_busy") or 0.0)
    return "texture path (TA/TD)" if td > (pmc.get("valu_busy") or 0.0) + 0.1 else "valu"


def roofline_of(alg_bytes, ms):
    achieved = alg_bytes / (ms * 1e-3) / 1e9
    return achieved, achieved / HBM_PEAK_GBPS


def lane_utils(s):
    """Wave-loop lane utilisations from the STATS counters (each <= 1)."""
    return {"primary": round(s["primary_fetches"] / max(1, 64 * s["primary_wave_iters"]), 4),
            "march": round(s["shadow_fetches"] / max(1, 64 * s["march_wave_iters"]), 4),
            "march_marching_lanes": round(s["shadow_fetches"] / max(1, s["march_lane_slots"]), 4),
            "how": "fetches / (64 x wave loop iterations); march_marching_lanes: over the lanes that began "
                   "each march (idle lanes of sky / unlit pixels excluded)"}


# ---------------------------------------------------------------- N > 1
def multi_rank(args, torch, dist, vx, scene, frame, W, H, K, rank, world, local, standin):
    """Bands dealt round-robin, rendered in place, gathered to rank 0; timed max over ranks."""
    from voxmap_amd.dist import band_rows_for, rows_per_rank
    BAND = band_rows_for(H, world)      # the band height whose deal loads the busiest rank least
    dev = "cpu" if standin else "cuda"
    sync = (lambda: None) if standin else torch.cuda.synchronize
    mg = split_ms = None
    if standin:
        streams = [None] * K
    else:
        streams = [torch.cuda.Stream() for _ in range(K)]
        torch.cuda.set_stream(streams[0])
    frames = [torch.empty((H, W, 4), dtype=torch.uint8, device=dev) for _ in range(K)]
    group = None
    gather = args.gather
    gloo = gather == "gloo" and not standin
    if standin or gloo:
        gather = "torch"
    elif gather == "native":
        uid = [vx.mgpu_unique_id() if rank == 0 else None]
        dist.broadcast_object_list(uid, src=0)
        try:
            mg = vx.MultiGPU(scene, uid[0], world, rank)
            ok = torch.tensor([1])
        except Exception as e:          # RCCL init refused: fall back to the torch-driven gather
            print(f"rank {rank}: vx_mgpu_create failed ({e}); falling back to --gather torch", file=sys.stderr)
            mg, ok = None, torch.tensor([0])
        dist.all_reduce(ok, op=dist.ReduceOp.MIN)
        if int(ok.item()) == 0:
            if mg is not None:
                mg.close()
                mg = None
            gather = "torch-fallback"
            group = dist.new_group(list(range(world)), backend="nccl")
    if gather == "native":
        fns = [(lambda fb=frames[j], sj=streams[j].cuda_stream:
                mg.render(frame, BAND, fb.data_ptr(), pixel_format=vx.PIXEL_RGBA8, stream=sj)) for j in range(K)]
        st = mg.render(frame, BAND, frames[0].data_ptr(), pixel_format=vx.PIXEL_RGBA8,
                       stream=streams[0].cuda_stream, stats=True).as_dict()
        gather_desc = "vx_mgpu_render: one RCCL ncclSend/ncclRecv group into rank 0's frame rows (native C++)"
    else:
        from voxmap_amd.dist import BandGather, band_rows_of
        gs = []
        for j in range(K):
            if standin:
                def rb(ids, fr, j=j):                  # stand-in renderer: each band filled from its id
                    for b in ids:
                        fr[band_rows_of(b, H, BAND)] = (b * 7 + j) % 251
            elif gloo:
                def rb(ids, fr, j=j, sj=streams[j]):  # render on the GPU, bands to host for gloo
                    scene.render_bands(frame, BAND, ids, frames[j].data_ptr(), inplace=True, stream=sj.cuda_stream)
                    sj.synchronize()
                    for b in ids:
                        r = band_rows_of(b, H, BAND)
                        fr[r] = frames[j][r].cpu()
            else:
                def rb(ids, fr, sj=streams[j].cuda_stream):
                    scene.render_bands(frame, BAND, ids, fr.data_ptr(), inplace=True, stream=sj)
            g = BandGather(dist, W, H, BAND, 4, torch.uint8, "cpu" if gloo else dev, rb, group=group)
            if not gloo:
                g.frame = frames[j]
            gs.append(g)

        def mk(j):
            def f():
                if standin or gloo:
                    gs[j].step()
                else:
                    with torch.cuda.stream(streams[j]):
                        gs[j].step()
            return f
        fns = [mk(j) for j in range(K)]
        if standin:
            gs[0].step()
            st = {"pixels": W * sum(band_rows_of(b, H, BAND).stop - band_rows_of(b, H, BAND).start
                                    for b in gs[0].mine), "shadow_rays": 0, "reflect_rays": 0, "alg_bytes": 0,
                  "kernel_ms": 0.0}
        else:
            st = scene.render_bands(frame, BAND, gs[0].mine, frames[0].data_ptr(), inplace=True,
                                    stream=streams[0].cuda_stream, stats=True).as_dict()
        gather_desc = ("torch.distributed batch_isend_irecv into rank 0's frame rows" +
                       (" (fallback: vx_mgpu_create failed)" if group is not None else "") +
                       (" (gloo, CPU stand-in renderer)" if standin else
                        " (gloo through host memory: one-GPU rehearsal, not a timing)" if gloo else " (RCCL)"))
    keys = [k for k in st.keys() if k != "kernel_ms"]
    vec = torch.tensor([float(st[k]) for k in keys], dtype=torch.float64)
    on_dev = gather == "torch" and not standin and not gloo
    if on_dev:
        vec = vec.cuda()
    dist.all_reduce(vec)
    stats = {k: float(v) for k, v in zip(keys, vec.cpu().tolist())}
    stats["kernel_ms"] = float(st["kernel_ms"])
    n = [0]

    def step():
        fns[n[0] % K]()
        n[0] += 1
    walls, settle_steps = timed(sync, step, args.steps, args.warmup, 0.0 if standin else args.settle_ms, dist,
                                "cuda" if on_dev else None, repeats=REPEATS)
    tt = torch.tensor(walls, dtype=torch.float64)
    if on_dev:
        tt = tt.cuda()
    dist.all_reduce(tt, op=dist.ReduceOp.MAX)             # per block, the slowest rank
    med, blocks = block_summary([float(v) for v in tt.cpu().tolist()], args.steps)
    wall = med * args.steps / 1000.0
    if gloo:
        # the rehearsal's check: rank 0's gathered frame == one whole-frame render
        j_last = (n[0] - 1) % K
        if rank == 0:
            full = torch.empty((H, W, 4), dtype=torch.uint8, device="cuda")
            scene.render_device(frame, full.data_ptr(), pixel_format=vx.PIXEL_RGBA8)
            torch.cuda.synchronize()
            stats["gather_frame_ok"] = bool(torch.equal(full.cpu(), gs[j_last].frame))
    if rank == 0 and standin:
        # the gathered frame must hold every band's stand-in value
        from voxmap_amd.dist import band_rows_of as bro
        j_last = (n[0] - 1) % K
        good = all(int(frames[j_last][bro(b, H, BAND)][0, 0, 0]) == (b * 7 + j_last) % 251
                   for b in range(-(-H // BAND)))
        stats["standin_frame_ok"] = bool(good)
    # render and gather timed apart (one stream, one frame at a
    # time, max over ranks): this rank's bands rendered alone (vx_render_bands),
    # then the gather alone (collective: vx_mgpu_gather, or BandGather.gather
    # on the torch / stand-in path)
    try:
        if mg is not None:
            mine = vx.mgpu_bands(H, BAND, world, rank)
            s0 = streams[0].cuda_stream

            def r_only():
                if mine:
                    scene.render_bands(frame, BAND, mine, frames[0].data_ptr(), inplace=True, stream=s0)

            def g_only():
                mg.gather(W, H, BAND, frames[0].data_ptr(), stream=s0)
            gbytes = int(sum(x[5] for x in vx.mgpu_transfers(W, H, BAND, world, 0)))
        else:
            def r_only():
                if standin or gloo:
                    gs[0].render()
                else:
                    with torch.cuda.stream(streams[0]):
                        gs[0].render()

            def g_only():
                if standin or gloo:
                    gs[0].gather()
                else:
                    with torch.cuda.stream(streams[0]):
                        gs[0].gather()
            from voxmap_amd.dist import transfers as _tr
            gbytes = int(sum(x[5] for x in _tr(W, H, BAND, world, 0, 4)))
        tr, _ = timed(sync, r_only, args.steps, 2, 0.0, dist, "cuda" if on_dev else None)
        tg, _ = timed(sync, g_only, args.steps, 2, 0.0, dist, "cuda" if on_dev else None)
        t2 = torch.tensor([tr[0], tg[0]], dtype=torch.float64)
        if on_dev:
            t2 = t2.cuda()
        dist.all_reduce(t2, op=dist.ReduceOp.MAX)
        t2 = t2.cpu()
        split_ms = {"render_ms": round(1000.0 * float(t2[0]) / args.steps, 4),
                    "gather_ms": round(1000.0 * float(t2[1]) / args.steps, 4),
                    "gather_bytes": gbytes,
                    "how": "one stream, one frame at a time, max over ranks (the timed step overlaps "
                           "frames in flight, so it is less than the sum)" +
                           ("; CPU stand-in renderer, gloo gather" if standin else "")}
    except Exception as e:                # never let the diagnostic break the bench line
        split_ms = {"error": str(e)}
    if mg is not None:
        mg.close()
    rpr = rows_per_rank(H, BAND, world)
    shards = {"unit": f"{BAND}-row full-width bands", "count": -(-H // BAND),
              "rows_per_rank_max_over_mean": round(max(rpr) / (sum(rpr) / world), 5),
              "assignment": "round-robin (band b -> rank b % N)", "gather": gather_desc, "split_ms": split_ms}
    return stats, wall, settle_steps, shards, blocks


# ---------------------------------------------------------------- main
def main(argv=None):
    argv = sys.argv[1:] if argv is None else argv
    args = parse(argv)
    if args.gpus > 1 and "WORLD_SIZE" not in os.environ:
        return spawn_ranks(args.gpus, argv)
    import torch
    import torch.distributed as dist

    world = max(int(os.environ.get("WORLD_SIZE", "1")), 1)
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if args.gather == "gloo":                  # one-GPU rehearsal: every rank on this device
        local = int(os.environ.get("VOXMAP_BENCH_DEVICE", str(local)))
    standin = args.standin
    if world > 1:
        # native gather: RCCL lives in libvoxmap_hip.so; torch.distributed (gloo) only
        # shares the RCCL unique id, holds the barriers and takes the max time
        if args.gather == "torch" and not standin:
            torch.cuda.set_device(local)
            dist.init_process_group("nccl", device_id=torch.device("cuda", local))
        else:
            dist.init_process_group("gloo")
    if not standin:
        torch.cuda.set_device(local)
    import voxmap_amd as vx
    from voxmap_amd import presets, scenes

    cfg_name = args.config or ("C3" if world == 1 else "C4")
    cfg = presets.CONFIGS[cfg_name]
    cam = args.camera or cfg["camera"]
    if cfg_name == "C4" or world == 1:
        W, H = cfg["w"], cfg["h"]
        scaling = "strong" if world > 1 else "weak"
    else:
        s = math.sqrt(world)
        W, H, scaling = int(round(cfg["w"] * s / 32)) * 32, int(round(cfg["h"] * s / 8)) * 8, "weak"
    if standin:
        W = min(W, 256)      # narrow frames; the full height keeps the config's band deal
    up = 3.0 if cfg["scene"] == "s_up3" else 1.0
    flags = args.flags if args.flags is not None else (vx.FLAG_FULL_QUALITY if args.quality == "full" else 0)
    samples = args.samples if args.samples is not None else cfg.get("samples", 1)
    frame = presets.camera_frame(cam, W, H, scale=up, flags=flags, shadow_samples=samples,
                                 sun_radius=args.sun_radius if samples > 1 else 0.0)
    K = max(1, args.inflight if args.inflight is not None else (4 if world == 1 else 2))

    X = Y = Z = 0
    t_scene = 0.0
    scene = noise = None
    if not standin:
        grid = presets.scene_grid(cfg["scene"])
        Z, Y, X = grid.shape
        noise = scenes.real_noise()            # the reference's res/noise.bin.gz (u_noise, render.js:138)
        t_scene = time.perf_counter()
        # palette grid in, distance field + octant copies built on the device (f-1);
        # the noise texture through the product's .gz loader
        scene = vx.Scene(map_bytes=grid.tobytes(), map_format=vx.FORMAT_GRID, noise_path=scenes.NOISE_PATH,
                         dims=(X, Y, Z), device=local)
        t_scene = time.perf_counter() - t_scene
        del grid

    shards = None
    exit_info = None
    if world == 1:
        r = single_gpu(torch, vx, scene, frame, W, H, K, args.steps, args.warmup, args.settle_ms)
        stats, wall, settle_steps, ev_ms = r["stats"], r["wall_s"], r["settle"], r["ev_ms"]
        exit_info, blocks = r["exit"], r["blocks"]
    else:
        stats, wall, settle_steps, shards, blocks = multi_rank(args, torch, dist, vx, scene, frame, W, H, K, rank,
                                                               world, local, standin)
        ev_ms = None
    ms_per_step = 1000.0 * wall / args.steps

    v1 = c5 = d2h = None
    if world == 1 and flags != 0 and args.flags is None and samples <= 1:
        # the reference's own shader (v1, flags 0) on the same frame: the same
        # K-in-flight wall timing, and one stream with events for its roofline
        fr1 = presets.camera_frame(cam, W, H, scale=up)
        a = single_gpu(torch, vx, scene, fr1, W, H, K, args.steps, args.warmup, 0.0, repeats=3)
        s1 = a["stats"]
        r1 = s1["pixels"] + s1["shadow_rays"]
        ms1w = 1000.0 * a["wall_s"] / args.steps
        v1 = {"ms_per_frame": round(ms1w, 4), "mrays_per_s": round(r1 / ms1w / 1e3, 3), "rays_per_frame": int(r1),
              "single_stream_ms_per_frame": round(a["ev_ms"], 4), "alg_bytes": int(s1["alg_bytes"]),
              "roofline_frac": round(roofline_of(s1["alg_bytes"], a["ev_ms"])[1], 4),
              "lane_util": lane_utils(s1), "exit_tables": a["exit"]}
    if world == 1 and not args.no_d2h:
        d2h = fps_with_d2h(torch, vx, scene, frame, W, H, max(20, args.steps // 2))
    if world == 1 and cfg_name == "C3" and not args.no_c5 and args.flags is None and args.samples is None:
        # BASELINE configs[4] in the same run (C5 next to C3)
        c5cfg = presets.CONFIGS["C5"]
        g5 = presets.scene_grid(c5cfg["scene"])
        Z5, Y5, X5 = g5.shape
        t5 = time.perf_counter()
        sc5 = vx.Scene(map_bytes=g5.tobytes(), map_format=vx.FORMAT_GRID, noise_path=scenes.NOISE_PATH,
                       dims=(X5, Y5, Z5), device=local)
        t5 = time.perf_counter() - t5
        del g5
        f5 = presets.camera_frame(c5cfg["camera"], c5cfg["w"], c5cfg["h"], scale=3.0, flags=flags,
                                  shadow_samples=c5cfg["samples"], sun_radius=args.sun_radius)
        n5 = max(10, args.steps // 5)
        b = single_gpu(torch, vx, sc5, f5, c5cfg["w"], c5cfg["h"], K, n5, 3, 100.0, repeats=3)
        s5 = b["stats"]
        rays5 = s5["pixels"] + s5["shadow_rays"] + s5["reflect_rays"]
        marched5 = rays5 - s5["shadow_rays_resolved"]
        ms5 = 1000.0 * b["wall_s"] / n5
        ach5, frac5 = roofline_of(s5["alg_bytes"], b["ev_ms"])
        # the same frame's bytes without the sun doom table (DESIGN.md §3 "Doom table":
        # the table skips fetches of marches that end unlit anyway, so the frame's own
        # bytes fall with its time); that march's bytes over this frame's time
        f5n = vx.Frame(f5.params.copy(), c5cfg["w"], c5cfg["h"])
        f5n.params.flags |= vx.FLAG_NO_DOOM
        o5 = torch.empty(c5cfg["w"] * c5cfg["h"] * 4, dtype=torch.uint8, device="cuda")
        torch.cuda.synchronize()
        s5n = sc5.render_device(f5n, o5.data_ptr(), pixel_format=vx.PIXEL_RGBA8, stats=True).as_dict()
        torch.cuda.synchronize()
        del o5
        frac5n = roofline_of(s5n["alg_bytes"], b["ev_ms"])[1]
        t5j = pmc_entry(f"traffic_{PMC_TAG}_c5.json", "C5", c5cfg["camera"], flags, c5cfg["samples"])
        c5 = {"workload": f"C5: {c5cfg['w']}x{c5cfg['h']}, field {X5}x{Y5}x{Z5} (S-proc 3x nearest upsample), "
                          f"full quality + {c5cfg['samples']}-sample soft shadows (sun radius {args.sun_radius})",
              "ms_per_frame": round(ms5, 4), "fps": round(1000 / ms5, 2),
              # a soft-shadowed fragment whose first step lands in a marked exit-table block
              # resolves all its samples by one table test: those rays are
              # resolved, not marched
              "mrays_per_s_resolved": round(rays5 / ms5 / 1e3, 3), "rays_resolved_per_frame": int(rays5),
              "mrays_per_s_marched": round(marched5 / ms5 / 1e3, 3), "rays_marched_per_frame": int(marched5),
              "single_stream_ms_per_frame": round(b["ev_ms"], 4),
              "alg_bytes": int(s5["alg_bytes"]), "roofline_achieved_gbps": round(ach5, 2),
              "roofline_frac": round(frac5, 4), "traffic": t5j.get("hbm_bytes_per_launch") if t5j else None,
              "alg_bytes_no_doom": int(s5n["alg_bytes"]), "roofline_frac_no_doom_bytes": round(frac5n, 4),
              "lane_util": lane_utils(s5), "scene_build_s": round(t5, 3), "frames": n5, "timing": b["blocks"],
              "exit_tables": b["exit"]}
        sc5.close()
    c3ra = None
    if world == 1 and cfg_name == "C3" and flags == vx.FLAG_FULL_QUALITY and args.flags is None and samples <= 1:
        # a reflection workload over the whole frame -- every first
        # surface traces its mirror ray (VX_FLAG_REFLECT_ALL), next to the headline
        fra = presets.camera_frame(cam, W, H, scale=up, flags=flags | vx.FLAG_REFLECT_ALL)
        c = single_gpu(torch, vx, scene, fra, W, H, K, args.steps, args.warmup, 0.0, repeats=3)
        sr = c["stats"]
        rr = sr["pixels"] + sr["shadow_rays"] + sr["reflect_rays"]
        msr = 1000.0 * c["wall_s"] / args.steps
        c3ra = {"workload": "C3 full quality + VX_FLAG_REFLECT_ALL (every first surface mirrors the traced scene, "
                            "Schlick-weighted; DESIGN.md §3 Extensions)",
                "ms_per_frame": round(msr, 4), "mrays_per_s": round(rr / msr / 1e3, 3), "rays_per_frame": int(rr),
                "reflect_rays": int(sr["reflect_rays"]), "single_stream_ms_per_frame": round(c["ev_ms"], 4),
                "alg_bytes": int(sr["alg_bytes"]), "roofline_frac": round(roofline_of(sr["alg_bytes"], c["ev_ms"])[1], 4),
                "timing": c["blocks"]}

    # rays per frame: primary + shadow + reflection rays resolved.  With soft
    # shadows some shadow rays are settled by one exit-table test of the
    # fragment's first step (shadow_rays_resolved) instead of a
    # march; rays_marched_per_frame / mrays_per_s_marched count only the marched ones
    rays = stats["pixels"] + stats["shadow_rays"] + stats["reflect_rays"]
    marched = rays - stats.get("shadow_rays_resolved", 0)
    value = rays * args.steps / wall / 1e6                                   # whole-job Mrays/s
    result = None
    if rank == 0:
        per_launch_bytes = float(stats["alg_bytes"]) / world if world > 1 else float(stats["alg_bytes"])
        kernel_ms = ev_ms if world == 1 else stats["kernel_ms"]
        achieved, frac = roofline_of(per_launch_bytes, kernel_ms) if kernel_ms else (0.0, 0.0)
        tag = PMC_TAG if cfg_name != "C5" else f"{PMC_TAG}_c5"
        traffic = pmc_entry(f"traffic_{tag}.json", cfg_name, cam, flags, samples) if world == 1 else None
        valu = pmc_entry(f"valu_{tag}.json", cfg_name, cam, flags, samples) if world == 1 else None
        if valu is None and not standin:
            # the same kernel instantiation measured on another workload (C2/C4 and
            # every rank of N > 1 run the C3 kernel; soft shadows the C5 one)
            ref_cfg = "C5" if samples > 1 else "C3"
            c_ref = presets.CONFIGS[ref_cfg]
            valu = pmc_entry(f"valu_{PMC_TAG}{'_c5' if samples > 1 else ''}.json", ref_cfg, c_ref["camera"], flags,
                             c_ref.get("samples", 1) if samples > 1 else 1)
            if valu is not None:
                valu = dict(valu, source=f"{valu.get('source', '')}; measured on {ref_cfg}, the same kernel "
                                         f"instantiation as this {cfg_name} run")
        result = {
            "metric": f"Mrays/s at {cfg['w']}x{cfg['h']} {'full quality' if flags else 'v1 shading'} "
                      f"({cfg_name}); fps; % HBM roofline",
            "value": round(value, 3),
            "unit": "Mrays/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(ms_per_step, 4),
            "higher_is_better": True,
            "scaling": scaling,
            "vs_baseline": None,
            "dtype": "fp32",
            "data": ("stand-in CPU band renderer (orchestration test, no GPU)" if standin else
                     f"synthetic {cfg['scene']} field (seed 1) in map.bin layout (the real map.blob is "
                     "AES-encrypted, key not in the repo); the reference's own res/noise.bin.gz noise texture"),
            "config": {
                "workload": f"{cfg_name}: {W}x{H} frame, " + (
                    "full quality = v1 shading (primary visibility + sun march + trilinear AO + sky/clouds + glass) "
                    "+ ext reflection + rough normals" if flags == vx.FLAG_FULL_QUALITY else
                    f"v1 shading flags={flags}") +
                    (f" + {samples}-sample soft shadows (sun radius {args.sun_radius})" if samples > 1 else "") +
                    f", field {X}x{Y}x{Z}, camera {cam}, sun hour 1.0, RGBA8 framebuffer in HBM",
                "value_is": (f"rays per second (primary + shadow + reflection; rays_marched_per_frame excludes soft-shadow rays settled by the first-step table test) over {K} frames in flight ({K} streams, {K} framebuffers), "
                             "inputs and framebuffers HBM-resident; the roofline uses the one-stream launch time"
                             if world == 1 else
                             f"rays marched per second by all {world} ranks, the RCCL gather to rank 0 inside "
                             f"each step, {K} frames in flight"),
                "flags": flags, "shadow_samples": samples, "scene_build_s": round(t_scene, 3),
                "clock_settle": {"ms": args.settle_ms, "untimed_frames": settle_steps},
                "timing": blocks,
                "width": W, "height": H, "field": [X, Y, Z], "camera": cam,
                "shards": shards,
                "fps": round(1000.0 / ms_per_step, 2),
                "fps_with_d2h": d2h,
                "inflight": {"frames": K, "streams": K, "framebuffers": K,
                             "single_stream_ms_per_frame": round(ev_ms, 4) if ev_ms is not None else None},
                "rays_per_frame": int(rays), "rays_marched_per_frame": int(marched),
                "mrays_per_s_marched": round(marched * args.steps / wall / 1e6, 3), "primary_rays": int(stats["pixels"]),
                "shadow_rays": int(stats["shadow_rays"]), "reflect_rays": int(stats["reflect_rays"]),
                "lane_util": lane_utils(stats) if world == 1 else None,
                "exit_tables": exit_info,
                "mrays_per_s_nominal_2rpp": round(2 * stats["pixels"] * args.steps / wall / 1e6, 3),
                "v1": v1,
                "c5": c5,
                "c3_reflect_all": c3ra,
                # not a roofline fraction: the reference's march takes every step of
                # render.frag:92-136 (VX_FLAG_NO_EXIT); the build's exit tables skip the
                # steps of marches that can no longer end unlit.  Work ratio of the same
                # frame in SURVEY §8d bytes (reference / this build); C5's is in c5.exit_tables.
                "reference_work_ratio": (round(exit_info["reference_alg_bytes"] / max(1, stats["alg_bytes"]), 4)
                                         if exit_info else None),
            },
            "roofline": {
                # achieved/peak/frac: the contract's unit, algorithmic bytes
                # over the HBM peak, per launch on ONE stream.  "bound" is the resource
                # that measurably binds the kernel: VALU issue (valu block: rocprofv3 PMC
                # kept under profiles/), the field being cache-resident (traffic = fabric
                # bytes << algorithmic)
                "bound": bound_of(valu),
                "kernel": "k_render (fused primary visibility + shading + sun march" +
                          (" + reflection walk" if flags & vx.FLAG_REFLECT else "") + ")",
                "achieved": round(achieved, 2),
                "peak": HBM_PEAK_GBPS,
                "unit": "GB/s",
                "frac": round(frac, 4),
                "traffic": traffic.get("hbm_bytes_per_launch") if traffic else None,
                "alg_bytes_per_launch": int(per_launch_bytes),
                "avg_launch_ms": round(kernel_ms, 4) if kernel_ms else None,
                "fabric_gbps": (round(traffic["hbm_bytes_per_launch"] / (kernel_ms * 1e-3) / 1e9, 1)
                                if traffic else None),
                "valu": ({k: valu[k] for k in ("valu_busy", "valu_lane_util", "valu_insts_per_wave", "clock_ghz",
                                               "source") if k in valu} if valu else None),
                "texture_path": ({k: valu[k] for k in ("ta_busy", "td_busy") if valu.get(k) is not None}
                                 if valu else None),
            },
        }
        if standin:
            result["config"]["standin_frame_ok"] = stats.get("standin_frame_ok")
        if "gather_frame_ok" in stats:
            result["config"]["gather_frame_ok"] = stats["gather_frame_ok"]
        if world == 1 and not args.no_cpu:
            result["cpu_baseline"] = cpu_baseline(scene, noise, frame, W, H, args.cpu_seconds)
    if scene is not None:
        scene.close()
    if world > 1:
        dist.barrier()
        dist.destroy_process_group()
    if rank == 0:
        print(json.dumps(result), flush=True)
    return 0


def host_cores():
    """(threads used, cores this process may run on, the node's hardware_concurrency).
    The GPU box allots a 1-GPU job 16 host cores (OMP_NUM_THREADS=16 there;
    os.cpu_count() shows the whole node): the baseline uses the allotment."""
    node = os.cpu_count() or 1
    try:
        aff = len(os.sched_getaffinity(0))
    except Exception:  # pragma: no cover
        aff = node
    omp = int(os.environ.get("OMP_NUM_THREADS", "0") or 0)
    return (max(1, min(omp, aff)) if omp > 0 else aff), aff, node


def cpu_baseline(scene, noise, frame, W, H, target_s):
    """The scalar oracle (oracle/, -O2 -fno-fast-math -ffp-contract=off, OpenMP
    over rows) on a bounded sample of the same frame: whole frames repeated
    until ~target_s when a frame is cheap (median rate reported), else a
    deterministic 1-in-k row subset sized to ~target_s; then the same on ONE
    core (a 1-in-k row subset of ~target_s/3)."""
    import numpy as np

    import oracle
    threads, aff, node = host_cores()
    field = scene.read_field()                # the map.bin bytes the GPU was given (R, G, B)
    o = oracle.Oracle(field, noise)
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
    # single core: a 1-in-k row subset of ~target_s/3
    k1 = 16
    t0 = time.perf_counter()
    _, st1 = o.render(frame.params, W, H, row0=k1 // 2, row_step=k1, threads=1, out=out)
    dt1 = time.perf_counter() - t0
    k1 = max(1, int(math.ceil(k1 * dt1 / max(target_s / 3, 1e-3))))
    t0 = time.perf_counter()
    _, st1 = o.render(frame.params, W, H, row0=k1 // 2, row_step=k1, threads=1, out=out)
    dt1 = time.perf_counter() - t0
    single = (st1.pixels + st1.shadow_rays + st1.reflect_rays) / dt1 / 1e6
    # the same frame by the oracle with this build's sun exit tables (the table
    # built once, outside the timing, as the GPU builds it once per sun window):
    # what the GPU's algorithm runs at on these cores
    same = None
    try:
        oe = oracle.Oracle(field, noise, exit=True)
        held = oe.hold_exit_table(frame.params)
        er = []
        t_end = time.perf_counter() + target_s / 3
        while time.perf_counter() < t_end or len(er) < 2:
            t0 = time.perf_counter()
            _, se = oe.render(frame.params, W, H, threads=threads, out=out)
            er.append((se.pixels + se.shadow_rays + se.reflect_rays) / (time.perf_counter() - t0) / 1e6)
            if len(er) >= 30:
                break
        same = {"value": round(float(np.median(er)), 4), "unit": "Mrays/s", "cores": threads,
                "sample": f"{len(er)} full {W}x{H} frames, median rate, exit table {held} held",
                "shadow_fetches": int(se.shadow_fetches)}
    except Exception as e:              # a diagnostic: never lose the baseline over it
        same = {"error": str(e)}
    return {
        "value": round(float(np.median(rates)), 4),
        "unit": "Mrays/s",
        "cores": threads,
        "kind": "port",
        "sample": desc,
        "single_core": {"value": round(single, 4), "unit": "Mrays/s", "cores": 1,
                        "sample": f"rows {k1 // 2}::{k1} of the same {W}x{H} frame ({st1.pixels} pixels) "
                                  f"in {dt1:.2f} s"},
        "same_algorithm": same,
        "host": {"threads_used": threads, "affinity_cores": aff, "hardware_concurrency": node,
                 "note": "the GPU box allots 16 host cores to a 1-GPU job (OMP_NUM_THREADS=16); "
                         "the oracle scales ~linearly over rows (independent pixels)"},
    }


if __name__ == "__main__":
    sys.exit(main())
