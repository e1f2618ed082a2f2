#!/bin/bash
# round 4: the head against the round-3 head (ab/lib_r03.so, built from git 69ca0cd)
# in one process: r03 ignores 0x800 (its split is the unit cell)
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$ROOT"; mkdir -p gpurun_out
timeout -k 10 400 python tools/abtime.py --config C3 --flags 48,2096,0,2048 --rounds 7 new=voxmap_amd/libvoxmap_hip.so r03=ab/lib_r03.so > gpurun_out/ab_r03_c3.txt 2>&1 || { echo "ab c3 failed"; tail gpurun_out/ab_r03_c3.txt; exit 1; }
cat gpurun_out/ab_r03_c3.txt
timeout -k 10 400 python tools/abtime.py --config C5 --flags 48 --rounds 3 --frames 10 new=voxmap_amd/libvoxmap_hip.so r03=ab/lib_r03.so > gpurun_out/ab_r03_c5.txt 2>&1 || { echo "ab c5 failed"; tail gpurun_out/ab_r03_c5.txt; exit 1; }
cat gpurun_out/ab_r03_c5.txt
