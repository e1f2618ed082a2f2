"""The multi-rank bench path on real hardware with one GPU (the
driver's 1/2/4/8-GPU runs need a node this repository never gets): bench.py
--gpus 2 --gather gloo spawns two ranks that both render on device 0 (RCCL
refuses two ranks on one device), deal the frame's bands, render them with the
HIP band kernel, move them over gloo through host memory into rank 0's frame,
and rank 0 checks the gathered frame against one whole-frame vx_render."""
import json
import os
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_two_ranks_on_one_gpu_gather_the_frame(built):
    try:
        import torch
        if not torch.cuda.is_available():
            pytest.skip("no GPU visible")
    except Exception:  # pragma: no cover
        pytest.skip("no torch")
    env = dict(os.environ)
    for k in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT"):
        env.pop(k, None)
    env["VOXMAP_BENCH_DEVICE"] = "0"
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2", "--gather", "gloo",
                        "--config", "C4", "--steps", "2", "--warmup", "1", "--inflight", "2", "--settle-ms", "0"],
                       cwd=ROOT, env=env, capture_output=True, text=True, timeout=240)
    assert r.returncode == 0, r.stderr[-3000:]
    lines = [l for l in r.stdout.splitlines() if l.startswith("{")]
    assert len(lines) == 1, r.stdout[-2000:]
    j = json.loads(lines[0])
    assert j["n_gpus"] == 2 and j["config"]["workload"].startswith("C4")
    assert j["config"]["gather_frame_ok"] is True          # every band in rank 0's frame, bit for bit
    sh = j["config"]["shards"]
    assert "gloo" in sh["gather"] and sh["rows_per_rank_max_over_mean"] <= 1.01
    assert sh["split_ms"]["render_ms"] > 0 and sh["split_ms"]["gather_ms"] > 0, sh["split_ms"]
