"""Screen-space sharding of one frame across GPUs — the
host-side mirror of the native path (vx_mgpu_*, csrc/vx_mgpu.cpp).

Pixels are independent (render.frag reads only the replicated field and noise
textures), so a frame is cut into full-width bands of ``band_rows`` rows,
dealt round-robin (band b -> rank b % world; neighbouring bands cost about the
same, so the interleave balances cheap sky against expensive geometry).  Every
rank renders its bands in place in its own w x h frame; rank 0 receives every
other rank's bands straight into the same rows of its frame with one batch of
point-to-point transfers.  A band is contiguous in a row-major frame, so there
is no tile-major staging buffer, no concatenation and no de-tile pass.

``BandGather`` runs that protocol over torch.distributed (gloo in the CPU
tests, "nccl" = RCCL with ``bench.py --gather torch``); the product path for
GPUs is the native vx_mgpu_render (bench.py default), which issues the same
transfers as one RCCL group from C++.
"""
from __future__ import annotations


def n_bands(h: int, band_rows: int) -> int:
    return -(-h // band_rows)


def bands(h: int, band_rows: int, world: int, rank: int) -> list:
    """Band ids of ``rank`` (vx_mgpu_bands): b = rank, rank + world, ..."""
    return list(range(rank, n_bands(h, band_rows), world))


def band_rows_for(h: int, world: int, max_rows: int = 64) -> int:
    """The deal's band height (vx_mgpu_band_rows): the multiple of 8 up to
    max_rows whose round-robin deal gives the busiest rank the fewest rows,
    ties to the tallest band (the fewest sends)."""
    if max_rows <= 0:
        max_rows = 64                   # as vx_mgpu_band_rows
    best, best_rows = 8, None
    for r in range(8, max(8, max_rows - max_rows % 8) + 1, 8):
        nb = n_bands(h, r)
        busiest = max(sum(min(h, (b + 1) * r) - b * r for b in range(k, nb, world)) for k in range(min(world, nb)))
        if best_rows is None or busiest <= best_rows:
            best, best_rows = r, busiest
    return best


def rows_per_rank(h: int, band_rows: int, world: int) -> list:
    return [sum(min(h, (b + 1) * band_rows) - b * band_rows for b in bands(h, band_rows, world, k))
            for k in range(world)]


def band_rows_of(b: int, h: int, band_rows: int) -> slice:
    return slice(b * band_rows, min(h, (b + 1) * band_rows))


def transfers(w: int, h: int, band_rows: int, world: int, rank: int, pixel_bytes: int) -> list:
    """The gather's point-to-point moves as ``rank`` issues them (the mirror of
    vx_mgpu_transfers): (band, src, dst, rows, byte offset, bytes) for every band
    whose owner is not rank 0 -- all of them on rank 0 (receives), the rank's own
    elsewhere (sends), in band order."""
    out = []
    for b in range(n_bands(h, band_rows)):
        owner = b % world
        if owner == 0 or (rank != 0 and owner != rank):
            continue
        r = band_rows_of(b, h, band_rows)
        rows = r.stop - r.start
        out.append((b, owner, 0, rows, r.start * w * pixel_bytes, rows * w * pixel_bytes))
    return out


class BandGather:
    """One rank's part of a sharded frame: render my bands in place, gather to rank 0.

    ``render_bands(ids, frame)`` is injected: on GPUs Scene.render_bands(inplace=True)
    into the frame tensor; CPU tests pass a host stand-in.  ``dist`` is an
    initialised torch.distributed.
    """

    def __init__(self, dist, w: int, h: int, band_rows: int, channels: int, dtype, device, render_bands, group=None):
        import torch
        self.dist = dist
        self.group = group
        self.world = dist.get_world_size()
        self.rank = dist.get_rank()
        self.w, self.h, self.band_rows = w, h, band_rows
        self.mine = bands(h, band_rows, self.world, self.rank)
        self.frame = torch.empty((h, w, channels), dtype=dtype, device=device)
        self._render = render_bands

    def transfers(self):
        """This rank's moves of the gather (``transfers``; the native vx_mgpu_transfers)."""
        px = self.frame.element_size() * self.frame.shape[2]
        return transfers(self.w, self.h, self.band_rows, self.world, self.rank, px)

    def step(self):
        self.render()
        return self.gather()

    def render(self):
        """My bands, in place in my frame."""
        if self.mine:
            self._render(self.mine, self.frame)

    def gather(self):
        """Every other rank's bands into rank 0's frame rows (collective)."""
        ops = []
        for b, src, dst, _, _, _ in self.transfers():
            rows = self.frame[band_rows_of(b, self.h, self.band_rows)]
            if self.rank == 0:
                ops.append(self.dist.P2POp(self.dist.irecv, rows, src, self.group))
            else:
                ops.append(self.dist.P2POp(self.dist.isend, rows, dst, self.group))
        if ops:
            for req in self.dist.batch_isend_irecv(ops):
                req.wait()
        return self.frame if self.rank == 0 else None
