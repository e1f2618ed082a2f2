"""The C++ host (voxmap_amd/vxrender, csrc/vx_cli.cpp) over the C ABI: it must
produce the same RGBA8 frame as the Python mirror for the same scene and
camera, from a palette grid and from an encrypted .blob (air written as B = 22
the way sdf.cpp writes map.bin, or as 0: identical frames)."""
import gzip
import json
import os
import subprocess

import numpy as np
import pytest

from voxmap_amd import _abi

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CLI = os.path.join(ROOT, "voxmap_amd", "vxrender")
KEY = "q83vEjRWeJCrze8SNFZ4kKvN7xI0VniQq83vEjRWeJA"   # test key (not the reference's)


def test_cli_help_and_errors(built):
    r = subprocess.run([CLI, "--help"], capture_output=True, text=True, timeout=60)
    assert r.returncode == 0 and f"ABI version {_abi.ABI_VERSION}" in r.stdout
    r = subprocess.run([CLI, "--map", "/nonexistent/map.bin"], capture_output=True, text=True, timeout=60)
    assert r.returncode == 2 and "cannot open" in r.stderr
    r = subprocess.run([CLI, "--bogus"], capture_output=True, text=True, timeout=60)
    assert r.returncode == 2


@pytest.mark.gpu
@pytest.mark.parametrize("source", ["grid", "blob", "blob_air0"])
def test_cli_frame_equals_python_host(built, tmp_path, source):
    import torch
    if not torch.cuda.is_available():
        pytest.skip("no GPU visible")
    import voxmap_amd as vx
    from voxmap_amd import presets, scenes
    dims = (128, 64, 24)
    grid = scenes.small_proc(11, dims=dims, n_boxes=16, n_glass=8)
    w, h = 320, 200
    sbj, rot = (64.0, 32.0, 20.0), (1.1, 0.0, 0.6)
    if source == "grid":
        path = tmp_path / "map.grid"
        path.write_bytes(grid.tobytes())
        extra = ["--format", "grid"]
    else:
        field = vx.field_build(grid)                 # air = B 22 (sdf.cpp:229-233)
        if source == "blob_air0":                    # the same map with air written as 0
            field[..., 2][grid == 0] = 0
        path = tmp_path / "map.blob"
        path.write_bytes(vx.blob_encrypt(gzip.compress(field.tobytes()), KEY))
        extra = ["--key", KEY]
    out = tmp_path / "frame.rgba"
    r = subprocess.run([CLI, "--map", str(path), *extra, "--dims", ",".join(map(str, dims)), "--size", f"{w},{h}",
                        "--orbit", ",".join(map(str, (*sbj, *rot))), "--full", "--frames", "3", "--out", str(out)],
                       capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stderr
    info = json.loads(r.stdout.strip().splitlines()[-1])
    assert info["size"] == [w, h] and info["ms_per_frame"] > 0
    img = np.frombuffer(out.read_bytes(), np.uint8).reshape(h, w, 4)
    fr = vx.make_frame(sbj, rot, w, h, hour=presets.SUN_HOUR, time=presets.TIME, flags=vx.FLAG_FULL_QUALITY)
    with vx.Scene(map_bytes=grid.tobytes(), map_format=vx.FORMAT_GRID, dims=dims, device=0) as sc:
        want, _ = sc.render(fr, pixel_format=vx.PIXEL_RGBA8)
    assert np.array_equal(img, want)


@pytest.mark.gpu
def test_cli_ranks_one_frame_equals_python_host(built, tmp_path):
    """vxrender --ranks 1: the forked rank process, the RCCL id through the pipe,
    vx_mgpu_create / vx_mgpu_render (this box has one GPU; N ranks need N GPUs)."""
    import torch
    if not torch.cuda.is_available():
        pytest.skip("no GPU visible")
    import voxmap_amd as vx
    from voxmap_amd import presets, scenes
    dims = (128, 64, 24)
    grid = scenes.small_proc(11, dims=dims, n_boxes=16, n_glass=8)
    w, h = 320, 200
    sbj, rot = (64.0, 32.0, 14.0), (1.2, 0.0, 2.0)
    path = tmp_path / "map.grid"
    path.write_bytes(grid.tobytes())
    out = tmp_path / "frame.rgba"
    r = subprocess.run([CLI, "--map", str(path), "--format", "grid", "--dims", ",".join(map(str, dims)),
                        "--size", f"{w},{h}", "--orbit", ",".join(map(str, (*sbj, *rot))), "--full", "--frames", "2",
                        "--ranks", "1", "--out", str(out)], capture_output=True, text=True, timeout=180)
    assert r.returncode == 0, r.stderr
    info = json.loads(r.stdout.strip().splitlines()[-1])
    assert info["ranks"] == 1 and info["rank0_pixels"] == w * h
    img = np.frombuffer(out.read_bytes(), np.uint8).reshape(h, w, 4)
    fr = vx.make_frame(sbj, rot, w, h, hour=presets.SUN_HOUR, time=presets.TIME, flags=vx.FLAG_FULL_QUALITY)
    with vx.Scene(map_bytes=grid.tobytes(), map_format=vx.FORMAT_GRID, dims=dims, device=0) as sc:
        want, _ = sc.render(fr, pixel_format=vx.PIXEL_RGBA8)
    assert np.array_equal(img, want)
