#!/bin/bash
# round 3: interleaved A/B of variant libraries (no parity run): C3 v1 + full, C5
# usage: bash tools/runs/r03_ab2.sh label=ab/lib.so ...   (ab/lib_base.so is always first)
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/../.." && pwd)}"
cd "$ROOT"; mkdir -p gpurun_out
timeout -k 10 300 python tools/abtime.py --config C3 --flags 0,48 --rounds 9 base=ab/lib_base.so "$@" > gpurun_out/ab2_c3.txt 2>&1 || { echo "ab c3 failed"; tail gpurun_out/ab2_c3.txt; exit 1; }
cat gpurun_out/ab2_c3.txt
timeout -k 10 300 python tools/abtime.py --config C5 --flags 48 --rounds 5 --frames 10 base=ab/lib_base.so "$@" > gpurun_out/ab2_c5.txt 2>&1 || { echo "ab c5 failed"; tail gpurun_out/ab2_c5.txt; exit 1; }
cat gpurun_out/ab2_c5.txt
