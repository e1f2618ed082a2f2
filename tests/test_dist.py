"""Screen-space sharding across ranks on CPU with gloo (voxmap_amd/dist.py, the
mirror of the native vx_mgpu_* protocol): band deal, in-place band render,
point-to-point gather into rank 0's frame rows.  The band renderer is a CPU
stand-in (rows cut from an oracle frame); on GPUs the same protocol runs in
C++ over RCCL (vx_mgpu_render, tests/test_parity_gpu.py at one rank, bench.py
at N ranks), and its deal is vx_mgpu_bands (checked against the mirror here)."""
import os
import socket

import numpy as np
import pytest


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _frame():
    import oracle
    import voxmap_amd as vx
    from voxmap_amd import scenes
    g = scenes.small_proc(9, dims=(64, 40, 12), n_boxes=10, n_glass=2)
    field = vx.field_build(g)
    noise = np.full((16, 16, 4), 100, np.uint8)
    fr = vx.make_frame((32.0, 20.0, 14.0), (1.0, 0.0, 0.4), 100, 70)
    img, _ = oracle.Oracle(field, noise).render(fr.params, 100, 70)
    return img


def _worker(rank, world, port, band_rows, q, inflight=1, rounds=1):
    import torch
    import torch.distributed as dist

    from voxmap_amd.dist import BandGather, band_rows_of
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        base = _frame()
        H, W = base.shape[:2]

        def context(img):
            def render_bands(ids, frame):
                for b in ids:
                    rows = band_rows_of(b, H, band_rows)
                    frame[rows] = torch.from_numpy(img[rows])
            g = BandGather(dist, W, H, band_rows, 4, torch.float32, "cpu", render_bands)
            g.frame.fill_(float("nan"))       # rows rank 0 neither renders nor receives would show
            return g

        # frames in flight (bench.py --inflight): one BandGather per in-flight
        # frame, each with its own frame and content, stepped alternately
        imgs = [base + np.float32(j) for j in range(inflight)]
        ctxs = [context(im) for im in imgs]
        ok = True
        for i in range(rounds * inflight):
            j = i % inflight
            out = ctxs[j].step()
            if rank == 0:
                ok &= bool(np.array_equal(out.numpy().view(np.uint32), imgs[j].view(np.uint32)))
        if rank == 0:
            q.put(ok)
    finally:
        dist.destroy_process_group()


def _run(world, band_rows, inflight=1, rounds=1):
    import torch.multiprocessing as mp
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, band_rows, q, inflight, rounds)) for r in range(world)]
    for p in procs:
        p.start()
    for p in procs:
        p.join(timeout=180)
    assert all(p.exitcode == 0 for p in procs), [p.exitcode for p in procs]
    assert q.get(timeout=5) is True


@pytest.mark.parametrize("world,band_rows", [(2, 8), (3, 16), (5, 8), (2, 64)])
def test_band_gather_gloo(built, world, band_rows):
    """Ragged last band (70 rows), more ranks than some deals, one band per rank."""
    _run(world, band_rows)


def test_band_gather_frames_in_flight_gloo(built):
    """Two frames in flight (bench.py's double buffering for N > 1): two
    BandGathers stepped alternately keep their own frames."""
    _run(2, 16, inflight=2, rounds=3)


def test_band_deal_is_a_partition_and_matches_native(built):
    import voxmap_amd as vx
    from voxmap_amd.dist import bands, n_bands
    for h, br in ((4320, 64), (2160, 32), (70, 8), (8, 8), (6112, 64)):
        for world in (1, 2, 4, 7, 8):
            lists = [bands(h, br, world, r) for r in range(world)]
            flat = sorted(t for l in lists for t in l)
            assert flat == list(range(n_bands(h, br)))
            sizes = [len(l) for l in lists]
            assert max(sizes) - min(sizes) <= 1                      # balanced to one band
            for r in range(world):
                assert vx.mgpu_bands(h, br, world, r) == lists[r]    # the native deal (vx_mgpu_bands)


@pytest.mark.parametrize("fmt,px", [(1, 4), (0, 16)])
def test_gather_schedule_native_matches_mirror(built, fmt, px):
    """vx_mgpu_transfers (what vx_mgpu_gather issues as one RCCL group) equals the
    mirror's schedule for N = 1..8, ragged last bands and both pixel formats; every
    send has its matching receive on rank 0, and rank 0's own bands plus what it
    receives tile the frame exactly once."""
    import voxmap_amd as vx
    from voxmap_amd.dist import bands, transfers
    for w, h, br in ((7680, 4320, 64), (3840, 2160, 64), (100, 70, 8), (64, 8, 8), (4096, 6112, 64), (33, 1000, 24)):
        for world in range(1, 9):
            sched = [vx.mgpu_transfers(w, h, br, world, r, fmt) for r in range(world)]
            for r in range(world):
                assert sched[r] == transfers(w, h, br, world, r, px), (w, h, br, world, r)
            recv = sched[0]
            sends = sorted(x for r in range(1, world) for x in sched[r])
            assert sends == recv                                       # one matching send per receive
            assert all(x[1] == x[0] % world and x[2] == 0 for x in recv)
            covered = np.zeros(h, np.int32)
            for b in bands(h, br, world, 0):
                covered[b * br:min(h, (b + 1) * br)] += 1
            for b, src, dst, rows, off, nbytes in recv:
                assert off == b * br * w * px and nbytes == rows * w * px
                covered[off // (w * px):off // (w * px) + rows] += 1
            assert (covered == 1).all(), (w, h, br, world)


def test_gather_schedule_rejects_bad_arguments(built):
    import voxmap_amd as vx
    for args in ((0, 8, 8, 2, 0, 1), (8, 8, 8, 2, 2, 1), (8, 8, 0, 2, 0, 1), (8, 8, 8, 2, 0, 7)):
        with pytest.raises(vx.VoxmapError):
            vx.mgpu_transfers(*args[:5], pixel_format=args[5])


def test_band_height_balances_the_deal(built):
    """vx_mgpu_band_rows: the band height whose round-robin
    deal loads the busiest rank least.  C4 (7680x4320) over 8 GPUs: 64-row
    bands gave ranks 576 or 512 rows (max/mean 1.067, a 93.75 % efficiency
    ceiling); the chosen 32-row bands give at most 544 (max/mean <= 1.01).
    The native choice equals the mirror's for every frame height and rank count."""
    import voxmap_amd as vx
    from voxmap_amd.dist import band_rows_for, rows_per_rank
    r = vx.mgpu_band_rows(4320, 8)
    rows = rows_per_rank(4320, r, 8)
    assert sum(rows) == 4320 and max(rows) / (4320 / 8) <= 1.01, (r, rows)
    assert max(rows_per_rank(4320, 64, 8)) == 576
    for h in list(range(8, 6200, 53)) + [1080, 2160, 3054, 4320, 6109]:
        for n in range(1, 9):
            b = vx.mgpu_band_rows(h, n)
            assert b == band_rows_for(h, n) and b % 8 == 0 and 8 <= b <= 64
            rp = rows_per_rank(h, b, n)
            assert sum(rp) == h
            # never worse than the fixed 64-row deal
            assert max(rp) <= max(rows_per_rank(h, 64, n))
    assert vx.mgpu_band_rows(4320, 8, 16) in (8, 16)
    # max_rows <= 0 means the default 64 on both sides
    for h, n in ((4320, 8), (2160, 3), (1000, 5)):
        for m in (0, -8):
            assert vx.mgpu_band_rows(h, n, m) == band_rows_for(h, n, m) == band_rows_for(h, n), (h, n, m)
