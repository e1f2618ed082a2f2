#!/bin/bash
# round 6: the GPU suite (optionally a -k filter in $K) and smoke() on the head
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/../.." && pwd)}"
cd "$ROOT"; mkdir -p gpurun_out
T=${TAG:-r06}
if [ -n "$K" ]; then SEL=(-k "$K"); else SEL=(); fi
timeout -k 10 1100 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread "${SEL[@]}" > gpurun_out/gpu_tests_$T.log 2>&1 || { echo "gpu tests failed rc=$?"; grep -E "FAILED|Error|passed|failed" gpurun_out/gpu_tests_$T.log | tail -20; exit 1; }
tail -2 gpurun_out/gpu_tests_$T.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke_$T.log 2>&1 || { echo "smoke failed"; tail -20 gpurun_out/smoke_$T.log; exit 1; }
tail -1 gpurun_out/smoke_$T.log
