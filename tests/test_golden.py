"""Golden frames (tests/golden/frames.npz, made by tests/golden/make_golden.py):
the oracle must reproduce them bit for bit (CPU), and so must the HIP path (GPU)."""
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


@pytest.mark.parametrize("case", META, ids=[c["name"] for c in META])
def test_oracle_reproduces_golden(built, case):
    import oracle
    mg = _load()
    field, noise, fr = mg.inputs(case)
    assert mg.sha(field) == case["field_sha256"], "field builder output changed"
    assert mg.sha(noise) == case["noise_sha256"], "synthetic noise changed"
    img, st = oracle.Oracle(field, noise).render(fr.params, case["w"], case["h"])
    gold = np.load(os.path.join(HERE, "frames.npz"))[case["name"]]
    assert np.array_equal(img.view(np.uint32), gold.view(np.uint32))
    assert st.as_dict() == case["stats"]


@pytest.mark.gpu
@pytest.mark.parametrize("case", META, ids=[c["name"] for c in META])
def test_hip_reproduces_golden(built, case):
    import torch
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    import voxmap_amd as vx
    mg = _load()
    field, noise, fr = mg.inputs(case)
    X, Y, Z = case["dims"]
    with vx.Scene(map_bytes=field.tobytes(), map_format=vx.FORMAT_BIN, noise_bytes=noise.tobytes(),
                  noise_format=vx.FORMAT_BIN, dims=(X, Y, Z), device=0) as sc:
        dev = sc.read_field()
        assert np.array_equal(dev[..., :3], field[..., :3])
        img, st = sc.render(fr, stats=True)
    gold = np.load(os.path.join(HERE, "frames.npz"))[case["name"]]
    assert np.array_equal(img.view(np.uint32), gold.view(np.uint32))
    for k, v in case["stats"].items():
        assert getattr(st, k) == v, k
