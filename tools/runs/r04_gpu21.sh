#!/bin/bash
# round 4, end: EXT 5/6 at 5 waves/SIMD -- GPU suite, smoke, the EXT 0/1
# kernels before and after the k_render / k_render_gen split (same box), bench
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/../.." && pwd)}"
cd "$ROOT"; mkdir -p gpurun_out
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/gpu_tests_r04e.log 2>&1 || { echo "gpu tests failed rc=$?"; grep -E "FAILED|Error|passed|failed" gpurun_out/gpu_tests_r04e.log | tail -20; exit 1; }
tail -2 gpurun_out/gpu_tests_r04e.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke_r04e.log 2>&1 || { echo "smoke failed"; tail -20 gpurun_out/smoke_r04e.log; exit 1; }
tail -1 gpurun_out/smoke_r04e.log
timeout -k 10 500 python tools/abtime.py --config C3 --flags 48,0 --rounds 7 presplit=ab/lean_presplit.so cur=ab/lean_cur.so > gpurun_out/ab_split_c3.txt 2>&1 || { echo "ab failed"; tail gpurun_out/ab_split_c3.txt; exit 1; }
cat gpurun_out/ab_split_c3.txt
timeout -k 10 900 python -u bench.py > gpurun_out/bench_r04_end2.jsonl 2> gpurun_out/bench_r04_end2.err || { echo "bench failed rc=$?"; tail -20 gpurun_out/bench_r04_end2.err; exit 1; }
python - <<'PY'
import json
d = json.loads(open("gpurun_out/bench_r04_end2.jsonl").read().strip().splitlines()[-1]); c = d["config"]
print(d["value"], d["ms_per_step"], "single", c["inflight"]["single_stream_ms_per_frame"], "v1", c["v1"]["ms_per_frame"],
      c["v1"]["single_stream_ms_per_frame"], "c5", c["c5"]["ms_per_frame"], c["c5"]["single_stream_ms_per_frame"],
      c["c5"]["roofline_frac"], "frac", d["roofline"]["frac"], "refl", c["c3_reflect_all"]["single_stream_ms_per_frame"])
PY
