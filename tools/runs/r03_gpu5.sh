#!/bin/bash
# round 3: TD micro (tools/micro/td_rate), then the parity subset + A/B of the current build
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/../.." && pwd)}"
cd "$ROOT"; mkdir -p gpurun_out
timeout -k 10 120 tools/micro/td_rate > gpurun_out/td_rate.txt 2>&1 || { echo "td_rate failed"; cat gpurun_out/td_rate.txt; exit 1; }
cat gpurun_out/td_rate.txt
AB_C5=1 bash tools/runs/r03_ab.sh
