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


def test_blend_stage_decides_bright_panes(built):
    """The GL blend stage (render.js:84-86 into the RGBA8 canvas of map.js:7;
    oracle blend_canvas): source, destination and alpha clamped to [0, 1], the
    destination read back as the canvas byte.  On 'blend_bright' (panes over
    cloudy sky brighter than 1 and grazing reflections) the round-5 fp32 blend
    (VXO_FLAG_BLEND_FLOAT) gives another frame, some pixels more than 1 LSB off;
    every other glass pixel moves by at most 1 LSB and nothing else moves."""
    import oracle
    mg = _load()
    case = next(c for c in META if c["name"] == "blend_bright")
    field, noise, fr, w, h = mg.inputs(case)
    O = oracle.Oracle(field, noise)
    new, st = O.render(fr.params, w, h)
    fr.params.flags |= mg.BLEND_FLOAT
    old, _ = O.render(fr.params, w, h)
    assert mg.sha(new) == case["frame_sha256"]
    assert mg.sha(old) == case["blend_float_sha256"]
    dq = np.abs(mg.quantise(new).astype(int) - mg.quantise(old).astype(int)).max(axis=2)
    assert int((dq > 0).sum()) == case["blend_float_differ_rgba8"]
    assert int((dq > 1).sum()) == case["blend_float_differ_over_1_lsb"] > 0
    changed = np.any(new.view(np.uint32) != old.view(np.uint32), axis=2)
    assert int(changed.sum()) <= st.glass_px          # only glass pixels blend
    # the new frame's glass pixels are the blend of clamped values: within [0, 1]
    assert float(new[changed][:, :3].max()) <= 1.0 and float(new[changed][:, :3].min()) >= 0.0
