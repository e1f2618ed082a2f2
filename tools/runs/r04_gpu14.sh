#!/bin/bash
# round 4: four frames in flight (bench value) with per-render cone reader
# events on every stream (head) against none (A/B variant), alternating runs
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/../.." && pwd)}"
cd "$ROOT"; mkdir -p gpurun_out
A="--no-cpu --no-c5 --no-d2h --steps 200 --warmup 20"
for r in 1 2; do
  timeout -k 10 300 python bench.py $A > gpurun_out/b_head_$r.json 2>/dev/null || { echo "bench head failed"; exit 1; }
  VOXMAP_LIB=ab/full_noevents.so timeout -k 10 300 python bench.py $A > gpurun_out/b_noev_$r.json 2>/dev/null || { echo "bench noev failed"; exit 1; }
done
python - <<'PY'
import json
for lab in ("head", "noev"):
    for r in (1, 2):
        d = json.loads(open(f"gpurun_out/b_{lab}_{r}.json").read().strip().splitlines()[-1])
        c = d["config"]
        print(lab, r, "ms/frame 4 in flight", d["ms_per_step"], "single", c["inflight"]["single_stream_ms_per_frame"],
              "v1", c["v1"]["ms_per_frame"], c["v1"]["single_stream_ms_per_frame"])
PY
