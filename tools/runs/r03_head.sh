#!/bin/bash
# round 3: the head on one MI355X -- smoke, every GPU test, the default bench
# line, then the rocprofv3 passes of C3 and C5 (tools/runs/r03_profile.sh).
# Each GPU step has its own time limit; the first failure ends the script.
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/../.." && pwd)}"
cd "$ROOT"; mkdir -p gpurun_out
timeout -k 10 180 python -c 'import __graft_entry__ as g; g.smoke()' > gpurun_out/smoke.log 2>&1 || { echo "smoke failed rc=$?"; tail -20 gpurun_out/smoke.log; exit 1; }
tail -2 gpurun_out/smoke.log
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1
rc=$?; tail -5 gpurun_out/pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python bench.py > gpurun_out/bench_head.jsonl 2> gpurun_out/bench_head.err || { echo "bench failed rc=$?"; tail -20 gpurun_out/bench_head.err; exit 1; }
cat gpurun_out/bench_head.jsonl
[ "${SKIP_PROF:-0}" = 1 ] || bash tools/runs/r03_profile.sh
