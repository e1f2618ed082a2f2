#!/bin/bash
# round 3: per-phase times of the head (abtime --flags: each VX_FLAG_* ablation of the same frame)
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/../.." && pwd)}"
cd "$ROOT"; mkdir -p gpurun_out
timeout -k 10 300 python tools/abtime.py --config C3 --flags 48,0,8,1,2,4,16,32,49,50,52 --rounds 5 new=voxmap_amd/libvoxmap_hip.so > gpurun_out/phases_c3.txt 2>&1 || { echo "phases failed"; tail gpurun_out/phases_c3.txt; exit 1; }
cat gpurun_out/phases_c3.txt
timeout -k 10 300 python tools/abtime.py --config C5 --flags 48,56,49,50,52 --rounds 3 --frames 10 new=voxmap_amd/libvoxmap_hip.so > gpurun_out/phases_c5.txt 2>&1 || { echo "phases c5 failed"; tail gpurun_out/phases_c5.txt; exit 1; }
cat gpurun_out/phases_c5.txt
