"""The built render kernels keep their occupancy and carry no KernelArgs copy
in scratch (voxmap_amd/kernel_meta.py).  CPU only: reads the
gfx950 code object's metadata out of the in-tree library."""
import pytest


@pytest.fixture(scope="module")
def meta(built):
    from voxmap_amd import build as vb
    from voxmap_amd import kernel_meta
    return kernel_meta.check(vb.OUT)


def _render(meta):
    from voxmap_amd import kernel_meta
    return {kernel_meta.render_params(k): v for k, v in meta.items() if kernel_meta.render_params(k)}


def test_every_render_instantiation_present(meta):
    # FMT 2 x STATS 2 x TILED 2 x (EXT modes 0-4 (v1, ext, soft, soft pooled, soft LDS bricks) x primary
    # index 2 + EXT 5-6 (glass in draw order, hard / soft shadows) x integer index only)
    assert len(_render(meta)) == 96


def test_render_kernels_fit_eight_waves_and_no_arg_copy(meta):
    from voxmap_amd import kernel_meta
    for p, v in _render(meta).items():
        lim = kernel_meta.STATS_SCRATCH_LIMIT if p[1] else kernel_meta.RENDER_SCRATCH_LIMIT
        assert v["private_segment_fixed_size"] <= lim, (p, v)
        if not p[1] and p[3] < 4:                      # timed (non-STATS) kernels
            assert v["vgpr_count"] <= 64 and v["sgpr_count"] <= 80, (p, v)
        elif not p[1] and p[3] >= 5:                   # EXT 5/6: their own budget (vx_render_e56.hip)
            assert v["vgpr_count"] <= kernel_meta.GENERAL_VGPR_LIMIT, (p, v)
        elif not p[1]:                                 # EXT 4: LDS bricks hold it to 7 waves/SIMD anyway
            assert v["vgpr_count"] <= 80, (p, v)


def test_product_kernels_spill_limits(meta):
    """The timed instantiations stay within their VGPR spill budgets (kernel_meta.SPILL_LIMITS)."""
    from voxmap_amd import kernel_meta
    for p, v in _render(meta).items():
        lim = kernel_meta.SPILL_LIMITS.get(p[3])
        if not p[1] and lim is not None:
            assert v["vgpr_spill_count"] <= lim, (p, v)


def test_no_spill_inside_a_step_loop(built):
    """No RGBA8 render kernel (every EXT mode) holds more spill instructions
    inside a march or primary step loop (kernel_meta.hot_loop_spills) than its
    mode allows: none, except the few reloads the doom rule's step loop takes
    in EXT 1/2/5 (kernel_meta.HOT_LOOP_SPILL_LIMITS, measured faster than the
    spill-free form); the rare paths (glass in draw order where panes stack)
    may spill, outside them."""
    from voxmap_amd import build as vb
    from voxmap_amd import kernel_meta
    hot = kernel_meta.hot_loop_spills(vb.OUT)
    assert len(hot) == 24, sorted(hot)
    for p, (loops, n) in hot.items():
        assert loops > 0 and n <= kernel_meta.HOT_LOOP_SPILL_LIMITS.get(p[3], 0), (p, loops, n)


def test_v1_kernel_main_path_spill_free(meta):
    """The reference shader's instantiations (EXT 0, not STATS) keep their
    registers: at most the stacked-glass chain's few spill slots, no KernelArgs copy."""
    from voxmap_amd import kernel_meta
    v1 = [v for p, v in _render(meta).items() if p[3] == 0 and p[1] == 0]
    assert len(v1) == 8
    assert all(v["vgpr_spill_count"] <= kernel_meta.SPILL_LIMITS[0] and
               v["private_segment_fixed_size"] <= kernel_meta.V1_SCRATCH_LIMIT for v in v1), [(v["vgpr_spill_count"], v["private_segment_fixed_size"]) for v in v1]
