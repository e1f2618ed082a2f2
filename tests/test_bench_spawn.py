"""bench.py's multi-GPU orchestration on CPU: ``python bench.py --gpus 2`` with no
launcher starts its own two rank processes (spawn_ranks: fresh interpreters,
torch.distributed.run's environment), which deal the frame's bands, gather them
into rank 0's frame (BandGather over gloo, the mirror of vx_mgpu_gather), take the
max time over ranks and print one JSON line.  --standin swaps the HIP band
renderer for a CPU stand-in; everything else is the path the 8-GPU run takes."""
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _bench(*args, timeout=240):
    env = dict(os.environ)
    for k in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT"):
        env.pop(k, None)
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), *args], cwd=ROOT, env=env,
                       capture_output=True, text=True, timeout=timeout)
    assert r.returncode == 0, r.stderr[-3000:]
    lines = [l for l in r.stdout.splitlines() if l.startswith("{")]
    assert len(lines) == 1, r.stdout
    return json.loads(lines[0])


def test_bench_spawns_its_own_ranks_gloo(built):
    j = _bench("--gpus", "2", "--standin", "--steps", "4", "--warmup", "1", "--inflight", "2")
    assert j["n_gpus"] == 2 and j["steps"] == 4 and j["warmup"] == 1
    assert j["scaling"] == "strong"                       # N > 1 defaults to C4 (7680x4320 for every N)
    assert j["config"]["workload"].startswith("C4")
    assert j["config"]["standin_frame_ok"] is True        # every band arrived in rank 0's frame
    sh = j["config"]["shards"]
    assert sh["assignment"].startswith("round-robin") and "gloo" in sh["gather"]
    assert j["value"] > 0 and j["ms_per_step"] > 0
    assert j["config"]["primary_rays"] == j["config"]["width"] * j["config"]["height"]


def test_bench_eight_ranks_standin_c4(built):
    """the driver's 8-GPU run rehearsed on CPU -- bench.py
    --gpus 8 spawns eight ranks, deals C4's 4320 rows (narrowed frames in the
    stand-in) in the band height vx_mgpu_band_rows picks, gathers over gloo and
    emits one line carrying the render / gather split and the deal's balance."""
    j = _bench("--gpus", "8", "--standin", "--steps", "3", "--warmup", "1", "--inflight", "2", timeout=600)
    assert j["n_gpus"] == 8 and j["steps"] == 3
    assert j["config"]["workload"].startswith("C4") and j["config"]["height"] == 4320
    assert j["config"]["standin_frame_ok"] is True
    sh = j["config"]["shards"]
    assert sh["unit"].startswith("32-row")                # vx_mgpu_band_rows(4320, 8)
    assert sh["rows_per_rank_max_over_mean"] <= 1.01
    sp = sh["split_ms"]
    assert sp["render_ms"] > 0 and sp["gather_ms"] > 0, sp
    assert sp["gather_bytes"] == j["config"]["width"] * 4 * (4320 - 544)   # all rows but rank 0's 544
