"""CPU tests of the C ABI (no GPU compute): symbols, error paths, codecs,
field builder parity with the literal restatements, camera/sun helpers."""
import gzip
import math
import os
import re
import shutil
import subprocess

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
REF = "/root/reference"


def test_library_exports_every_header_symbol(built):
    import voxmap_amd as vx
    from voxmap_amd import _abi
    header = open(os.path.join(ROOT, "include", "voxmap.h")).read()
    names = set(re.findall(r"^\s*(?:const\s+)?\w+\s*\*?\s*(vx_\w+)\s*\(", header, re.M))
    assert len(names) >= 15, names
    L = vx.lib()
    for n in names:
        assert hasattr(L, n), f"{n} missing from libvoxmap_hip.so"
    assert names == {s[0] for s in _abi.SIGNATURES}, names ^ {s[0] for s in _abi.SIGNATURES}
    assert L.vx_abi_version() == _abi.ABI_VERSION == 10


def test_error_paths_do_not_touch_the_gpu(built):
    import voxmap_amd as vx
    with pytest.raises(vx.VoxmapError) as e:
        vx.Scene(map_path="/nonexistent/map.bin")
    assert e.value.code == -2 and "cannot open" in str(e.value)
    with pytest.raises(vx.VoxmapError) as e:
        vx.Scene(map_bytes=b"\x00" * 100, map_format=vx.FORMAT_BIN, dims=(4, 4, 4))
    assert e.value.code == -5  # VX_ESIZE: 100 != 4*4*4*4
    with pytest.raises(vx.VoxmapError) as e:
        vx.Scene(map_bytes=b"\x00" * 256, map_format=vx.FORMAT_BIN, dims=(4, 4, 4), dist_cap=300)
    assert e.value.code == -1
    with pytest.raises(vx.VoxmapError) as e:
        vx.Scene(map_bytes=b"\xff" * 63, map_format=vx.FORMAT_GRID, dims=(4, 4, 4))
    assert e.value.code == -5
    with pytest.raises(vx.VoxmapError) as e:
        vx.decode(b"\x1f\x8bnot really gzip", vx.FORMAT_BIN_GZ)
    assert e.value.code == -3
    with pytest.raises(vx.VoxmapError) as e:
        vx.decode(b"\x00" * 17, vx.FORMAT_BLOB, key="A" * 43)
    assert e.value.code == -4


KEY = "q83vEjRWeJCrze8SNFZ4kKvN7xI0VniQq83vEjRWeJA"  # base64url of 32 test bytes (not a real key)


def test_jwk_key_decodes_to_32_bytes():
    import base64
    raw = base64.urlsafe_b64decode(KEY + "=")
    assert len(raw) == 32


def test_blob_round_trip_and_fixed_iv_against_openssl_cli(built, tmp_path):
    """.blob = AES-256-CBC(PKCS#7, fixed IV utils.js:11-16) of gzip bytes; checked
    against the independent openssl(1) implementation."""
    import base64

    import voxmap_amd as vx
    payload = gzip.compress(np.arange(5000, dtype=np.uint8).tobytes())
    blob = vx.blob_encrypt(payload, KEY)
    assert len(blob) % 16 == 0 and len(blob) > len(payload)
    assert vx.decode(blob, vx.FORMAT_BLOB, key=KEY) == np.arange(5000, dtype=np.uint8).tobytes()
    if not shutil.which("openssl"):
        pytest.skip("openssl CLI not available")
    key_hex = base64.urlsafe_b64decode(KEY + "=").hex()
    iv_hex = bytes([55, 44, 146, 89, 30, 93, 68, 30, 209, 23, 56, 140, 88, 149, 55, 221]).hex()
    src = tmp_path / "p.gz"
    src.write_bytes(payload)
    out = subprocess.run(["openssl", "enc", "-aes-256-cbc", "-K", key_hex, "-iv", iv_hex, "-in", str(src)],
                         check=True, capture_output=True).stdout
    assert out == blob
    with pytest.raises(vx.VoxmapError) as e:
        vx.decode(blob, vx.FORMAT_BLOB, key="B" + KEY[1:])
    assert e.value.code in (-3, -4)


@pytest.mark.skipif(not os.path.exists(f"{REF}/res/map.blob"), reason="reference assets absent")
def test_real_map_blob_size_pins_and_rejects_wrong_key(built):
    """res/map.blob: 543,824 B = 33,989 AES blocks; the key is not in
    the repository, so decoding with any test key must fail cleanly."""
    import voxmap_amd as vx
    blob = open(f"{REF}/res/map.blob", "rb").read()
    assert len(blob) == 543824 and len(blob) % 16 == 0
    assert open(f"{REF}/src/map.blob", "rb").read() == blob
    with pytest.raises(vx.VoxmapError) as e:
        vx.decode(blob, vx.FORMAT_BLOB, key=KEY)
    assert e.value.code in (-3, -4)


@pytest.mark.skipif(not os.path.exists(f"{REF}/res/noise.bin.gz"), reason="reference assets absent")
def test_real_noise_asset_decodes(built):
    """res/noise.bin.gz: 1024x1024 RGBA8 (render.js:141); A channel in 0..240, mean ~128."""
    import voxmap_amd as vx
    raw = vx.decode(open(f"{REF}/res/noise.bin.gz", "rb").read(), vx.FORMAT_BIN_GZ)
    assert len(raw) == 1024 * 1024 * 4
    a = np.frombuffer(raw, np.uint8).reshape(1024, 1024, 4)[..., 3]
    assert a.min() == 0 and a.max() == 240 and abs(a.mean() - 128.0) < 0.5


@pytest.mark.parametrize("dims,seed", [((1, 1, 1), 0), ((5, 1, 3), 1), ((3, 4, 5), 2), ((7, 6, 5), 3),
                                       ((9, 7, 6), 4), ((12, 10, 8), 5)])
def test_field_build_matches_pure_python_restatement(built, dims, seed):
    """vx_field_build and the C oracle against the line-by-line Python of sdf.cpp:405-470."""
    import oracle
    import voxmap_amd as vx
    from oracle import sdf_ref
    X, Y, Z = dims
    rng = np.random.default_rng(seed)
    g = (rng.random((Z, Y, X)) < 0.25).astype(np.uint8) * rng.integers(1, 22, (Z, Y, X)).astype(np.uint8)
    ref = sdf_ref.build(g)
    assert np.array_equal(oracle.field_build(g), ref)
    assert np.array_equal(vx.field_build(g), ref)


@pytest.mark.parametrize("seed", range(4))
def test_field_build_matches_oracle_mid_sizes(built, seed):
    import oracle
    import voxmap_amd as vx
    from voxmap_amd import scenes
    g = scenes.small_proc(seed + 100, dims=(80 + 8 * seed, 40, 12 + seed), n_boxes=12, n_glass=3)
    # include blocks in the 0-slices, where the clamped csum() quirk matters
    g[:, 0, ::7] = 4
    g[:, ::5, 0] = 9
    assert np.array_equal(vx.field_build(g, n_threads=4), oracle.field_build(g))


def test_field_build_full_size_matches_oracle(built):
    import oracle
    import voxmap_amd as vx
    from voxmap_amd import presets
    g = presets.scene_grid("s_proc")
    a = vx.field_build(g)
    assert a.shape == (32, 256, 1024, 4) and a.nbytes == 33554432     # map.bin size pin
    assert np.array_equal(a, oracle.field_build(g))
    assert not a[..., 3].any()                                           # sdf.cpp:469 writes A = 0
    assert (a[..., 2][g == 0] == 22).all()                               # air remapped to pal_size (:229-233)
    assert np.array_equal(a[..., 2][g != 0], g[g != 0])


def test_field_semantics_up_down():
    """R = 'up' half-cube radius (box [z, z+r]), G = 'down' (box [z-r, z]) (sdf.cpp:436-453)."""
    import voxmap_amd as vx
    g = np.zeros((8, 9, 9), np.uint8)
    g[0] = 1                       # ground
    g[6, 4, 4] = 3                 # a block above the centre column
    f = vx.field_build(g)
    # just below the floating block the up radius is 1 (box [5,6] contains it)
    assert f[5, 4, 4, 0] == 1
    # down radius of a ground-adjacent air cell is capped by max = z (sdf.cpp:437)
    assert f[1, 4, 4, 1] == 1
    assert f[3, 8, 8, 1] == 3
    assert (f[g > 0][:, :2] == 0).all()


def test_noise_synth_layout_and_determinism(built):
    import voxmap_amd as vx
    a, b = vx.noise_synth(0), vx.noise_synth(0)
    assert a.shape == (1024, 1024, 4) and np.array_equal(a, b)
    assert not np.array_equal(a, vx.noise_synth(1))
    alpha = a[..., 3].astype(float)
    assert 60 < alpha.mean() < 190 and alpha.std() > 5
    # tileable (REPEAT sampling, render.js:145-146): wrap-around steps are as smooth as interior ones
    d_wrap = np.abs(alpha[:, 0] - alpha[:, -1]).mean()
    d_in = np.abs(np.diff(alpha, axis=1)).mean()
    assert d_wrap < 3 * d_in + 1


def _js_camera(sbj, rot, w, h):
    """Independent numpy transcription of map.js:373-391 / math.js (column-major arrays)."""
    def mat(a):
        return np.array(a, dtype=np.float64).reshape(4, 4).T   # column-major -> row-major matrix
    def T(x, y, z):
        return mat([1, 0, 0, 0, 0, 1, 0, 0, 0, 0, 1, 0, x, y, z, 1])
    def Rx(t):
        c, s = math.cos(t), math.sin(t)
        return mat([1, 0, 0, 0, 0, c, s, 0, 0, -s, c, 0, 0, 0, 0, 1])
    def Rz(t):
        c, s = math.cos(t), math.sin(t)
        return mat([c, s, 0, 0, -s, c, 0, 0, 0, 0, 1, 0, 0, 0, 0, 1])
    def P(f, ratio, near, far):
        return mat([f / math.sqrt(ratio), 0, 0, 0, 0, f * math.sqrt(ratio), 0, 0, 0, 0, (near + far) / (near - far),
                    -1, 0, 0, 2 * near * far / (near - far), 0])
    orbit = T(*sbj) @ Rz(rot[2]) @ Rx(rot[0]) @ T(0, 0, sbj[2])
    pos = (orbit @ np.array([0, 0, 0, 1.0]))[:3]
    f = 1 / math.tan(60 * math.pi / 360)
    M = P(f, w / h, 1, 1024) @ Rx(-rot[0]) @ Rz(-rot[2]) @ T(*(-pos))
    return pos, M


@pytest.mark.parametrize("cam", ["K0", "K1", "K2"])
def test_orbit_camera_rays_project_to_their_pixels(built, cam):
    import voxmap_amd as vx
    from voxmap_amd import presets
    c = presets.CAMERAS[cam]
    w, h = 1920, 1080
    fr = vx.make_frame(c["sbj"], c["rot"], w, h)
    pos, M = _js_camera(c["sbj"], c["rot"], w, h)
    p = fr.params
    assert np.allclose(np.array(p.cam_cell) + np.array(p.cam_fract), pos, atol=1e-5)
    for px, py in [(0, 0), (w - 1, 0), (w // 3, h // 2), (w - 1, h - 1)]:
        nx = (2 * px + 1) / w - 1
        ny = 1 - (2 * py + 1) / h
        d = np.array(p.ray_fwd) + nx * np.array(p.ray_right) + ny * np.array(p.ray_up)
        clip = M @ np.append(pos + 50.0 * d, 1.0)
        assert clip[3] > 0
        assert abs(clip[0] / clip[3] - nx) < 1e-5 and abs(clip[1] / clip[3] - ny) < 1e-5


def test_frame_from_matrix_matches_orbit(built):
    import voxmap_amd as vx
    from voxmap_amd import presets
    c = presets.CAMERAS["K1"]
    pos, M = _js_camera(c["sbj"], c["rot"], 1280, 720)
    a = vx.make_frame(c["sbj"], c["rot"], 1280, 720).params
    col_major = M.T.reshape(-1).astype(np.float32)
    b = vx.frame_from_matrix(col_major, pos)
    for name in ("ray_fwd", "ray_right", "ray_up"):
        assert np.allclose(getattr(a, name), getattr(b, name), atol=2e-5), name
    assert list(a.cam_cell) == list(b.cam_cell)


def test_sun_from_hour():
    import voxmap_amd as vx
    s = vx.sun_from_hour(1.0)
    assert np.allclose(s, (0.7287352, 0.4207355, 0.5403023), atol=1e-6)
    assert abs(np.linalg.norm(s) - 1) < 1e-6


def test_scene_generators_deterministic():
    from voxmap_amd import scenes
    a, b = scenes.s_proc(1), scenes.s_proc(1)
    assert a.shape == (32, 256, 1024) and np.array_equal(a, b)
    assert (a == scenes.GLASS).any() and (a[0] > 0).all()
    assert set(np.unique(a)) <= set(range(22))
    c = scenes.s_campus()
    assert c.shape == (32, 256, 1024) and (c[0] > 0).all() and c[1:].any()
    assert scenes.upsample3(scenes.single_block()).shape == (48, 96, 192)


def test_offset_limits_rejected_before_any_upload(built):
    """the AO pair array (4 B per cell, X + 1 per row) and the noise
    quad planes (16 B per texel) use 32-bit byte offsets; fields and noise past
    them are refused by vx_scene_create's checks (no GPU touched)."""
    import voxmap_amd as vx
    with pytest.raises(vx.VoxmapError) as e:
        vx.Scene(map_bytes=b"\x00" * 64, map_format=vx.FORMAT_BIN, dims=(2048, 2100, 250))
    assert e.value.code == -1 and "4*(X+1)*Y*Z" in str(e.value)
    # just below the limit the same check passes (then the 64-byte map is the wrong size)
    with pytest.raises(vx.VoxmapError) as e:
        vx.Scene(map_bytes=b"\x00" * 64, map_format=vx.FORMAT_BIN, dims=(2048, 2040, 250))
    assert e.value.code == -5
    with pytest.raises(vx.VoxmapError) as e:
        vx.Scene(map_bytes=b"\x00" * 256, map_format=vx.FORMAT_BIN, dims=(4, 4, 4), noise_size=(16384, 16384))
    assert e.value.code == -1 and "noise too large" in str(e.value)
    with pytest.raises(vx.VoxmapError) as e:
        vx.Scene(map_bytes=b"\x00" * 256, map_format=vx.FORMAT_BIN, dims=(4, 4, 4), mesh_chunk=300)
    assert e.value.code == -1 and "mesh_chunk" in str(e.value)


def test_default_cap_falls_back_to_32_where_64_does_not_fit(built):
    """the default box cap (64) is also the octant copies' border;
    a field whose padded plane fits below 2^23 cells with 32 but not with 64
    (X = Y = 2800) is accepted with dist_cap = 0 (VX_FALLBACK_DIST_CAP), and
    refused only when 64 is asked for explicitly."""
    import voxmap_amd as vx
    dims = (2800, 2800, 4)
    grid = bytes(dims[0] * dims[1] * dims[2])
    with pytest.raises(vx.VoxmapError) as e:
        vx.Scene(map_bytes=grid, map_format=vx.FORMAT_GRID, dims=dims, dist_cap=64)
    assert e.value.code == -1 and "too large" in str(e.value)
    try:
        vx.Scene(map_bytes=grid, map_format=vx.FORMAT_GRID, dims=dims).close()   # a GPU: it loads
    except vx.VoxmapError as e2:                                                # no GPU: past validation
        assert e2.code != -1 and "too large" not in str(e2), str(e2)
