#!/bin/bash
# round 4: the full GPU suite and smoke() on the head
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/../.." && pwd)}"
cd "$ROOT"; mkdir -p gpurun_out
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/gpu_tests_r04.log 2>&1 || { echo "gpu tests failed rc=$?"; grep -E "FAILED|Error|passed|failed" gpurun_out/gpu_tests_r04.log | tail -20; exit 1; }
tail -3 gpurun_out/gpu_tests_r04.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke_r04.log 2>&1 || { echo "smoke failed"; tail -20 gpurun_out/smoke_r04.log; exit 1; }
tail -3 gpurun_out/smoke_r04.log
