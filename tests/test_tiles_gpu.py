"""Tiled launches at the edges of their grid shapes (vx_render.h launch_render_ext):
a tile list of more than 65535 tiles takes the 1-D grid, shorter lists the
(block columns, block rows, tiles) grid; a single one-block-row band, where both
shapes coincide; compact bands.  Every pixel equals the whole frame's."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu


def _gpu():
    try:
        import torch
        return torch.cuda.is_available()
    except Exception:  # pragma: no cover
        return False


@pytest.fixture(scope="module", autouse=True)
def _need_gpu(built):
    if not _gpu():
        pytest.skip("no GPU visible")


@pytest.fixture(scope="module")
def scene(noise):
    import voxmap_amd as vx
    from voxmap_amd import presets
    field = vx.field_build(presets.scene_grid("s_proc"))
    with vx.Scene(map_bytes=field.tobytes(), map_format=vx.FORMAT_BIN, noise_bytes=noise.tobytes(),
                  noise_format=vx.FORMAT_BIN, dims=(1024, 256, 32), device=0) as sc:
        yield sc


@pytest.mark.timeout(600)
@pytest.mark.parametrize("flags", [0, 48])
def test_more_than_65535_tiles_take_the_1d_grid(scene, flags):
    """8224 x 8192 in 32 x 32 tiles: 257 x 256 = 65792 tiles (the 1-D grid), every
    tile, detiled, equal to the whole frame; and the first 65535 of them (the
    3-D grid) equal to the same tiles."""
    import torch

    import voxmap_amd as vx
    from voxmap_amd import presets
    w, h, ts = 8224, 8192, 32
    fr = presets.camera_frame("K1", w, h, flags=flags)
    full = torch.zeros(w * h * 4, dtype=torch.uint8, device="cuda:0")
    torch.cuda.synchronize()            # the fill (torch's stream) before the scene's stream writes
    scene.render_device(fr, full.data_ptr(), pixel_format=vx.PIXEL_RGBA8)
    n = (w // ts) * (h // ts)
    assert n > 65535
    ids = list(range(n))
    tiles = torch.empty(n * ts * ts * 4, dtype=torch.uint8, device="cuda:0")
    scene.render_tiles(fr, ts, ids, tiles.data_ptr())
    frame = torch.zeros(w * h * 4, dtype=torch.uint8, device="cuda:0")
    torch.cuda.synchronize()
    scene.detile(w, h, ts, ids, tiles.data_ptr(), frame.data_ptr())
    torch.cuda.synchronize()
    assert torch.equal(frame, full)
    part = torch.empty(65535 * ts * ts * 4, dtype=torch.uint8, device="cuda:0")
    scene.render_tiles(fr, ts, ids[:65535], part.data_ptr())
    torch.cuda.synchronize()
    assert torch.equal(part, tiles[:part.numel()])


@pytest.mark.parametrize("inplace", [1, 0])
def test_single_block_row_bands_and_compact_bands(scene, inplace):
    """8-row bands (one block row each: a 1 x 1 tile-grid remainder in y), every
    third band, in place and compact, against the whole frame's rows."""
    import torch

    import voxmap_amd as vx
    from voxmap_amd import presets
    w, h = 1000, 600
    fr = presets.camera_frame("K1", w, h, flags=48)
    full, _ = scene.render(fr, pixel_format=vx.PIXEL_RGBA8)
    ids = list(range(0, h // 8, 3))
    for one in (ids, ids[:1]):
        out = torch.zeros((h if inplace else len(one) * 8) * w * 4, dtype=torch.uint8, device="cuda:0")
        torch.cuda.synchronize()        # the fill (torch's stream) before the scene's stream writes
        scene.render_bands(fr, 8, one, out.data_ptr(), inplace=bool(inplace), pixel_format=vx.PIXEL_RGBA8)
        torch.cuda.synchronize()
        img = out.cpu().numpy().reshape(-1, w, 4)
        for k, b in enumerate(one):
            got = img[8 * b:8 * b + 8] if inplace else img[8 * k:8 * k + 8]
            assert np.array_equal(got, full[8 * b:8 * b + 8]), (b, k)
