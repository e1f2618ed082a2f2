#!/bin/bash
# round 4: EXT 5/6 register budget -- 6 waves/SIMD (head) against 5 and 4
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/../.." && pwd)}"
cd "$ROOT"; mkdir -p gpurun_out
timeout -k 10 600 python tools/abtime.py --config C3 --flags 8240,4144 --rounds 5 --frames 10 gen6=voxmap_amd/libvoxmap_hip.so gen5=ab/full_gen5.so gen4=ab/full_gen4.so > gpurun_out/ab_gen2_c3.txt 2>&1 || { echo "ab failed"; tail gpurun_out/ab_gen2_c3.txt; exit 1; }
cat gpurun_out/ab_gen2_c3.txt
timeout -k 10 900 python -u bench.py > gpurun_out/bench_r04_end.jsonl 2> gpurun_out/bench_r04_end.err || { echo "bench failed rc=$?"; tail -20 gpurun_out/bench_r04_end.err; exit 1; }
python - <<'PY'
import json
d = json.loads(open("gpurun_out/bench_r04_end.jsonl").read().strip().splitlines()[-1]); c = d["config"]
print(d["value"], d["ms_per_step"], "single", c["inflight"]["single_stream_ms_per_frame"], "v1", c["v1"]["ms_per_frame"],
      c["v1"]["single_stream_ms_per_frame"], "c5", c["c5"]["ms_per_frame"], c["c5"]["single_stream_ms_per_frame"],
      c["c5"]["roofline_frac"], "frac", d["roofline"]["frac"], "refl", c["c3_reflect_all"]["single_stream_ms_per_frame"])
PY
