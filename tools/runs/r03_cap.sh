#!/bin/bash
# round 3: the primary traversal's box cap (scene dist_cap): 32 (default) vs 64 vs 128, same library
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/../.." && pwd)}"
cd "$ROOT"; mkdir -p gpurun_out
L=voxmap_amd/libvoxmap_hip.so
timeout -k 10 300 python tools/abtime.py --config C3 --flags 8,0,48 --rounds 7 c32=$L:32 c64=$L:64 c128=$L:128 > gpurun_out/cap_c3.txt 2>&1 || { echo "cap c3 failed"; tail gpurun_out/cap_c3.txt; exit 1; }
cat gpurun_out/cap_c3.txt
timeout -k 10 300 python tools/abtime.py --config C5 --flags 56,48 --rounds 3 --frames 10 c32=$L:32 c64=$L:64 > gpurun_out/cap_c5.txt 2>&1 || { echo "cap c5 failed"; tail gpurun_out/cap_c5.txt; exit 1; }
cat gpurun_out/cap_c5.txt
