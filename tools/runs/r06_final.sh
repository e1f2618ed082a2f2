#!/bin/bash
# round 6: rocprofv3 passes (tools/profile2.sh; summaries only are kept) for C3
# full quality, C5 and C3 + REFLECT_ALL, then the default bench line
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/../.." && pwd)}"
cd "$ROOT"; mkdir -p gpurun_out/r06_final
TAG=r06 BENCH_ARGS="--config C3" bash tools/profile2.sh || exit 1
TAG=r06_c5 BENCH_ARGS="--config C5" bash tools/profile2.sh || exit 1
TAG=r06_refl BENCH_ARGS="--config C3 --flags 8240" bash tools/profile2.sh || exit 1
cd "$ROOT"
python tools/prof_summary2.py r06 C3 K1 48 1 > gpurun_out/r06_final/summ_r06.log 2>&1 || { echo "summary failed"; tail gpurun_out/r06_final/summ_r06.log; exit 1; }
python tools/prof_summary2.py r06_c5 C5 K1 48 16 > gpurun_out/r06_final/summ_r06_c5.log 2>&1 || { echo "summary c5 failed"; tail gpurun_out/r06_final/summ_r06_c5.log; exit 1; }
python tools/prof_summary2.py r06_refl C3 K1 8240 1 > gpurun_out/r06_final/summ_r06_refl.log 2>&1 || { echo "summary refl failed"; tail gpurun_out/r06_final/summ_r06_refl.log; exit 1; }
for t in r06 r06_c5 r06_refl; do cp profiles/${t}_kernel_stats.csv profiles/${t}_pmc.json profiles/traffic_${t}.json profiles/valu_${t}.json gpurun_out/r06_final/; done
rm -rf gpurun_out/prof_r06 gpurun_out/prof_r06_c5 gpurun_out/prof_r06_refl
timeout -k 10 900 python -u bench.py > gpurun_out/r06_final/bench.jsonl 2> gpurun_out/r06_final/bench.err || { echo "bench failed rc=$?"; tail -20 gpurun_out/r06_final/bench.err; exit 1; }
python - <<'PY'
import json
d = json.loads(open("gpurun_out/r06_final/bench.jsonl").read().strip().splitlines()[-1]); c = d["config"]
print(d["value"], d["ms_per_step"], "single", c["inflight"]["single_stream_ms_per_frame"], "v1", c["v1"]["ms_per_frame"],
      c["v1"]["single_stream_ms_per_frame"], "c5", c["c5"]["ms_per_frame"], c["c5"]["single_stream_ms_per_frame"],
      c["c5"]["roofline_frac"], "frac", d["roofline"]["frac"], "refl", c["c3_reflect_all"]["single_stream_ms_per_frame"])
PY
