#!/bin/bash
# round 4: the bench line as the driver runs it (--steps 20 --warmup 5) and the
# default run, on the same box
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/../.." && pwd)}"
cd "$ROOT"; mkdir -p gpurun_out
timeout -k 10 900 python -u bench.py --steps 20 --warmup 5 > gpurun_out/bench_r04_s20.jsonl 2> gpurun_out/bench_r04_s20.err || { echo "bench s20 failed rc=$?"; tail -20 gpurun_out/bench_r04_s20.err; exit 1; }
timeout -k 10 900 python -u bench.py > gpurun_out/bench_r04_final.jsonl 2> gpurun_out/bench_r04_final.err || { echo "bench failed rc=$?"; tail -20 gpurun_out/bench_r04_final.err; exit 1; }
python - <<'PY'
import json
for f in ("gpurun_out/bench_r04_s20.jsonl", "gpurun_out/bench_r04_final.jsonl"):
    d = json.loads(open(f).read().strip().splitlines()[-1]); c = d["config"]
    print(f, d["value"], d["ms_per_step"], c["timing"]["ms_per_step_blocks"], "single", c["inflight"]["single_stream_ms_per_frame"],
          "c5", c["c5"]["single_stream_ms_per_frame"], c["c5"]["roofline_frac"], "frac", d["roofline"]["frac"])
PY
