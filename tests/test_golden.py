"""Golden frames (tests/golden/, made by tests/golden/make_golden.py; SURVEY §8c
item (5)): the oracle must reproduce them bit for bit (CPU), and so must the
HIP path (GPU).  Frames are compared by the SHA-256 of the fp32 RGBA bytes;
the stored pixels (fp32 for small frames, RGBA8 for 256x256) locate a mismatch."""
import json
import os

import numpy as np
import pytest

HERE = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")
META = json.load(open(os.path.join(HERE, "frames.json")))


def _load():
    import sys
    sys.path.insert(0, HERE)
    import make_golden
    return make_golden


_ORACLES = {}


def _check(mg, case, img):
    gold = np.load(os.path.join(HERE, "frames.npz"))[case["name"]]
    if mg.stored(case):
        bad = int(np.count_nonzero(img.view(np.uint32) != gold.view(np.uint32)))
    else:
        bad = int(np.count_nonzero(mg.quantise(img) != gold))
    assert mg.sha(img) == case["frame_sha256"], f"frame differs from the golden one ({bad} stored values differ)"
    assert bad == 0


@pytest.mark.parametrize("case", META, ids=[c["name"] for c in META])
def test_oracle_reproduces_golden(built, case):
    import oracle
    mg = _load()
    field, noise, fr, w, h = mg.inputs(case)
    assert mg.sha(field) == case["field_sha256"], "field builder output changed"
    assert mg.sha(noise) == case["noise_sha256"], "noise texture changed"
    key = case.get("scene") or case["name"]
    if key not in _ORACLES:
        _ORACLES.clear()
        _ORACLES[key] = oracle.Oracle(field, noise)
    img, st = _ORACLES[key].render(fr.params, w, h)
    _check(mg, case, img)
    assert st.as_dict() == case["stats"]


_EXIT = {}


def _exit_oracle(key, field, noise):
    import oracle
    if key not in _EXIT:
        _EXIT.clear()
        _EXIT[key] = oracle.Oracle(field, noise, exit=True)
    return _EXIT[key]


@pytest.mark.parametrize("case", META, ids=[c["name"] for c in META])
def test_oracle_exit_tables_keep_golden(built, case):
    """The build's sun exit tables change no pixel: the oracle
    marching with them reproduces every golden frame, with no more shadow
    fetches than the reference's literal march and every other counter equal."""
    mg = _load()
    field, noise, fr, w, h = mg.inputs(case)
    img, st = _exit_oracle(case.get("scene") or case["name"], field, noise).render(fr.params, w, h)
    _check(mg, case, img)
    d = st.as_dict()
    for k, v in case["stats"].items():
        if k == "shadow_fetches":
            assert d[k] <= v
        else:
            assert d[k] == v, k


@pytest.mark.gpu
@pytest.mark.parametrize("case", META, ids=[c["name"] for c in META])
def test_hip_reproduces_golden(built, case):
    import torch
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    import voxmap_amd as vx
    mg = _load()
    field, noise, fr, w, h = mg.inputs(case)
    Z, Y, X, _ = field.shape
    with vx.Scene(map_bytes=field.tobytes(), map_format=vx.FORMAT_BIN, noise_bytes=noise.tobytes(),
                  noise_format=vx.FORMAT_BIN, dims=(X, Y, Z), device=0) as sc:
        dev = sc.read_field()
        assert np.array_equal(dev[..., :3], field[..., :3])
        img, st = sc.render(fr, stats=True)                  # with the sun exit tables
        fr.params.flags |= vx.FLAG_NO_EXIT
        img_lit, st_lit = sc.render(fr, stats=True)          # every step of the reference's march
    _check(mg, case, img)
    _check(mg, case, img_lit)
    for k, v in case["stats"].items():
        assert getattr(st_lit, k) == v, k
    _, ost = _exit_oracle(case.get("scene") or case["name"], field, noise).render(fr.params, w, h)
    for k, v in ost.as_dict().items():
        assert getattr(st, k) == v, k
