#!/bin/bash
# round 5: the default bench line (N = 1); TAG names the output
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/../.." && pwd)}"
cd "$ROOT"; mkdir -p gpurun_out
T=${TAG:-r05}
timeout -k 10 900 python -u bench.py ${BENCH_ARGS} > gpurun_out/bench_$T.jsonl 2> gpurun_out/bench_$T.err || { echo "bench failed rc=$?"; tail -20 gpurun_out/bench_$T.err; exit 1; }
python - "$T" <<'PY'
import json, sys
d = json.loads(open(f"gpurun_out/bench_{sys.argv[1]}.jsonl").read().strip().splitlines()[-1]); c = d["config"]
print(d["value"], d["ms_per_step"], "single", c["inflight"]["single_stream_ms_per_frame"], "v1", c["v1"]["ms_per_frame"],
      c["v1"]["single_stream_ms_per_frame"], "c5", c["c5"]["ms_per_frame"], c["c5"]["single_stream_ms_per_frame"],
      c["c5"]["roofline_frac"], "frac", d["roofline"]["frac"], "refl", c["c3_reflect_all"]["single_stream_ms_per_frame"])
PY
