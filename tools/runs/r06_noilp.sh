#!/bin/bash
# round 6: EXT 0/1 without the max-ilp schedule (ab/noilp.so) against the head, now
# that the hard march carries the doom rule
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/../.." && pwd)}"
cd "$ROOT"; mkdir -p gpurun_out
L=voxmap_amd/libvoxmap_hip.so
timeout -k 10 400 python -u tools/abtime.py --config C3 --flags 48,0 --rounds 11 --frames 20 head=$L noilp=ab/noilp.so > gpurun_out/ab_noilp_c3.txt 2>&1 || { echo "c3 ab failed"; tail -20 gpurun_out/ab_noilp_c3.txt; exit 1; }
cat gpurun_out/ab_noilp_c3.txt
timeout -k 10 300 python -u tools/abtime.py --config C3 --scene s_glass --flags 48 --rounds 9 --frames 20 head=$L noilp=ab/noilp.so > gpurun_out/ab_noilp_glass.txt 2>&1 || { echo "glass ab failed"; tail -20 gpurun_out/ab_noilp_glass.txt; exit 1; }
cat gpurun_out/ab_noilp_glass.txt
