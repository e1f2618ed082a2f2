#!/bin/bash
# round 6: the doom table for the hard shadow too (ab/doom_hard.so) against the
# head (soft shadows only): C3 full quality and v1, S-glass
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/../.." && pwd)}"
cd "$ROOT"; mkdir -p gpurun_out
L=voxmap_amd/libvoxmap_hip.so
timeout -k 10 300 python -u tools/abtime.py --config C3 --flags 48,0 --rounds 9 --frames 20 head=$L hard=ab/doom_hard.so hardoff=ab/doom_hard.so+131072 > gpurun_out/ab_doom8_c3.txt 2>&1 || { echo "c3 ab failed"; tail -20 gpurun_out/ab_doom8_c3.txt; exit 1; }
cat gpurun_out/ab_doom8_c3.txt
timeout -k 10 300 python -u tools/abtime.py --config C3 --scene s_glass --flags 48 --rounds 9 --frames 20 head=$L hard=ab/doom_hard.so > gpurun_out/ab_doom8_glass.txt 2>&1 || { echo "glass ab failed"; tail -20 gpurun_out/ab_doom8_glass.txt; exit 1; }
cat gpurun_out/ab_doom8_glass.txt
