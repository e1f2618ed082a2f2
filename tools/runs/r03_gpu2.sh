#!/bin/bash
# round 3: GPU tests (full-frame parity) + one bench run of the head
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/../.." && pwd)}"
cd "$ROOT"; mkdir -p gpurun_out
timeout -k 10 180 python -c 'import __graft_entry__ as g; g.smoke()' > gpurun_out/smoke.log 2>&1 || { echo "smoke failed rc=$?"; tail -20 gpurun_out/smoke.log; exit 1; }
tail -2 gpurun_out/smoke.log
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 600 --timeout-method thread --durations=15 > gpurun_out/pytest_gpu.log 2>&1
rc=$?; tail -25 gpurun_out/pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python bench.py --steps 50 --warmup 5 > gpurun_out/bench.log 2>&1
rc=$?; tail -1 gpurun_out/bench.log; exit $rc
