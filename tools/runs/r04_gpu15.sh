#!/bin/bash
# round 4: no per-render reader events -- the GPU suite (two-thread sun
# cycling included) and the bench figures without CPU / C5 / D2H legs
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/../.." && pwd)}"
cd "$ROOT"; mkdir -p gpurun_out
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/gpu_tests_r04b.log 2>&1 || { echo "gpu tests failed rc=$?"; grep -E "FAILED|Error|passed|failed" gpurun_out/gpu_tests_r04b.log | tail -20; exit 1; }
tail -2 gpurun_out/gpu_tests_r04b.log
timeout -k 10 300 python bench.py --no-cpu --no-c5 --no-d2h --steps 200 --warmup 20 > gpurun_out/b_head3.json 2>/dev/null || { echo "bench failed"; exit 1; }
python -c "
import json
d=json.loads(open('gpurun_out/b_head3.json').read().strip().splitlines()[-1]); c=d['config']
print('4 in flight', d['ms_per_step'], 'single', c['inflight']['single_stream_ms_per_frame'], 'v1', c['v1']['ms_per_frame'], c['v1']['single_stream_ms_per_frame'])"
