"""Pins of the oracle's restatements against OUTPUTS the reference itself ships
(VERDICT r01 "what's weak" #3).

* res/vertex2d.bin.gz — the plaintext 2D mesh sdf.cpp:362-401 wrote for the
  real campus (tests/golden/vertex2d.bin.gz, a byte copy of the reference
  asset).  The restated mesher (oracle/mesh_ref.py mesh2d, vertex2d_bytes)
  regenerates it BYTE FOR BYTE from the footprint it encodes: greedy merge
  order, quad/triangle/record layout (sdf.cpp:154-173), glass id, and air
  (pal_size after the remap, sdf.cpp:229-239) never meshed.  Negative controls
  show the pin discriminates (a mesher that meshes air, or scans y-major, or
  swaps the triangle order, produces different bytes).
* res/noise.bin.gz — shipped as voxmap_amd/data/noise.bin.gz (used by the
  GPU tests and the bench as u_noise): SHA-256 of the file and of the
  decoded texture, texel spot checks, decoded by the product codec.
"""
import gzip
import hashlib
import os

import numpy as np
import pytest

HERE = os.path.dirname(os.path.abspath(__file__))
V2D = os.path.join(HERE, "golden", "vertex2d.bin.gz")
V2D_SHA = "e1a6ed3ad0e350577ec1e1ac6cd84596e6d469d559a726a1d0424e146ae226f3"
NOISE_GZ_SHA = "7e6ca94cfcb8ce582e7b93e803eab8ee7049202e9c20586ebc5fc00df3ca9253"
NOISE_RAW_SHA = "4bc5167887f4615ade0c7309959d378f0738c2646352fbe7512bcaa36f4d96a9"
NOISE_TEXELS = {(0, 0): [103, 198, 105, 219], (0, 1023): [190, 73, 14, 220], (511, 512): [67, 5, 137, 129],
                (1023, 0): [215, 190, 165, 221], (1023, 1023): [118, 151, 170, 221],
                (123, 456): [232, 192, 248, 194], (700, 33): [105, 221, 112, 111]}


@pytest.fixture(scope="module")
def v2d():
    blob = open(V2D, "rb").read()
    assert hashlib.sha256(blob).hexdigest() == V2D_SHA
    return gzip.decompress(blob)


def test_vertex2d_regenerated_byte_for_byte(v2d):
    from oracle import mesh_ref
    assert len(v2d) == 19116 * 16                          # 19,116 vertices of 16 B
    c2d = mesh_ref.decode_vertex2d(v2d)
    assert 22 in c2d and not (c2d == 0).any()             # uncovered = air = pal_size; 0 never occurs
    quads = mesh_ref.mesh2d(c2d)
    assert len(quads) == 19116 // 6
    assert mesh_ref.vertex2d_bytes(quads) == v2d


def test_vertex2d_pin_discriminates(v2d):
    """The regeneration is not a tautology: plausible misreadings of sdf.cpp give other bytes."""
    from oracle import mesh_ref
    c2d = mesh_ref.decode_vertex2d(v2d)
    # meshing air as well (a loop to colour <= pal_size)
    extra = mesh_ref.mesh2d(c2d, pal_size=23)
    assert mesh_ref.vertex2d_bytes([q[:5] + (0,) for q in extra]) != v2d
    # y-major scan (forYX instead of forXY) merges differently
    yq = mesh_ref.mesh2d(c2d.T.copy())
    yq = [(y, x, h, w, c, i) for (x, y, w, h, c, i) in yq]
    assert mesh_ref.vertex2d_bytes(yq) != v2d
    # the colours in the records are the remapped indices, glass id only for pal_size - 1
    rec = np.frombuffer(v2d, mesh_ref.REC2D)
    assert set(np.unique(rec["c"])) <= set(range(1, 22)) and ((rec["id"] == 2) == (rec["c"] == 21)).all()


def test_vertex_record_layout_3d():
    """vert() records of the 3D mesh (sdf.cpp:94-141): 16 B, six per quad,
    winding swapped for odd normals."""
    from oracle import mesh_ref
    q = np.array([[3, 4, 5, 2, 0, 0, 0, 0, 1, 7, 4, 0], [3, 4, 5, 2, 0, 0, 0, 0, 1, 7, 5, 0]], np.int32)
    rec = np.frombuffer(mesh_ref.vertex_bytes(q), mesh_ref.REC2D)
    assert len(rec) == 12
    assert rec["d"][:6].tolist() == [[0, 0, 0], [2, 0, 0], [0, 0, 1], [0, 0, 1], [2, 0, 0], [2, 0, 1]]
    assert rec["d"][6:].tolist() == [[0, 0, 0], [0, 0, 1], [2, 0, 0], [0, 0, 1], [2, 0, 1], [2, 0, 0]]
    assert (rec["n"] == [4] * 6 + [5] * 6).all() and (rec["c"] == 7).all()


def test_real_noise_fixture_checksums_and_texels(built):
    import voxmap_amd as vx
    from voxmap_amd import scenes
    blob = open(scenes.NOISE_PATH, "rb").read()
    assert hashlib.sha256(blob).hexdigest() == NOISE_GZ_SHA
    raw = vx.decode(blob, vx.FORMAT_BIN_GZ)                # the product codec
    assert hashlib.sha256(raw).hexdigest() == NOISE_RAW_SHA and raw == gzip.decompress(blob)
    a = np.frombuffer(raw, np.uint8).reshape(1024, 1024, 4)
    for (y, x), want in NOISE_TEXELS.items():
        assert a[y, x].tolist() == want, (y, x)
    assert a[..., 3].min() == 0 and a[..., 3].max() == 240 and abs(a[..., 3].mean() - 128.0) < 0.05
    assert np.array_equal(scenes.real_noise(), a)


@pytest.mark.skipif(not os.path.exists("/root/reference/res/noise.bin.gz"), reason="reference absent")
def test_fixtures_are_the_reference_assets():
    """In the build container: the shipped fixtures are byte copies of the reference's assets."""
    from voxmap_amd import scenes
    assert open(scenes.NOISE_PATH, "rb").read() == open("/root/reference/res/noise.bin.gz", "rb").read()
    assert open(V2D, "rb").read() == open("/root/reference/res/vertex2d.bin.gz", "rb").read()


def test_vertex2d_regenerated_from_the_campus_map(built, v2d):
    """End to end through the product's host code: S-campus as map.bin (the
    footprint extruded, air = B 22) -> vx_vertex2d (each column's top block,
    sdf.cpp:201-204, meshed by the C++ restatement of sdf.cpp:362-401) == the
    reference's vertex2d.bin byte for byte; the oracle's footprint + mesher too."""
    import oracle
    import voxmap_amd as vx
    from oracle import mesh_ref
    from voxmap_amd import presets
    field = vx.field_build(presets.scene_grid("s_campus"))
    assert vx.vertex2d(field) == v2d
    c = oracle.footprint(field)
    assert mesh_ref.vertex2d_bytes(mesh_ref.mesh2d(np.where(c == 0, 22, c).T.copy())) == v2d
