#!/bin/bash
# round 4, final head: rocprofv3 passes for C3 and C5 (tools/profile2.sh, summaries
# only are kept) and the default bench line
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/../.." && pwd)}"
cd "$ROOT"; mkdir -p gpurun_out
TAG=r04 BENCH_ARGS="--config C3" bash tools/profile2.sh || exit 1
TAG=r04_c5 BENCH_ARGS="--config C5" bash tools/profile2.sh || exit 1
cd "$ROOT"
python tools/prof_summary2.py r04 C3 K1 48 1 > gpurun_out/summ_r04.log 2>&1 || { echo "summary failed"; tail gpurun_out/summ_r04.log; exit 1; }
python tools/prof_summary2.py r04_c5 C5 K1 48 16 > gpurun_out/summ_r04_c5.log 2>&1 || { echo "summary c5 failed"; tail gpurun_out/summ_r04_c5.log; exit 1; }
mkdir -p gpurun_out/r04_final
cp profiles/r04_kernel_stats.csv profiles/r04_pmc.json profiles/traffic_r04.json profiles/valu_r04.json \
   profiles/r04_c5_kernel_stats.csv profiles/r04_c5_pmc.json profiles/traffic_r04_c5.json profiles/valu_r04_c5.json gpurun_out/r04_final/
rm -rf gpurun_out/prof_r04 gpurun_out/prof_r04_c5
timeout -k 10 900 python -u bench.py > gpurun_out/r04_final/bench.jsonl 2> gpurun_out/r04_final/bench.err || { echo "bench failed rc=$?"; tail -20 gpurun_out/r04_final/bench.err; exit 1; }
python - <<'PY'
import json
d = json.loads(open("gpurun_out/r04_final/bench.jsonl").read().strip().splitlines()[-1]); c = d["config"]
print(d["value"], d["ms_per_step"], "single", c["inflight"]["single_stream_ms_per_frame"], "v1", c["v1"]["ms_per_frame"],
      c["v1"]["single_stream_ms_per_frame"], "c5", c["c5"]["ms_per_frame"], c["c5"]["single_stream_ms_per_frame"],
      c["c5"]["roofline_frac"], "frac", d["roofline"]["frac"], "refl", c["c3_reflect_all"]["single_stream_ms_per_frame"])
PY
