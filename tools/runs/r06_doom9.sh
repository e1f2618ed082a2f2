#!/bin/bash
# round 6: the doom table for the hard shadow (ab/doom_hard.so) against the head,
# second pass: C3 full quality, v1, REFLECT_ALL; S-glass full quality
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/../.." && pwd)}"
cd "$ROOT"; mkdir -p gpurun_out
L=voxmap_amd/libvoxmap_hip.so
timeout -k 10 400 python -u tools/abtime.py --config C3 --flags 48,0,8240 --rounds 11 --frames 20 head=$L hard=ab/doom_hard.so > gpurun_out/ab_doom9_c3.txt 2>&1 || { echo "c3 ab failed"; tail -20 gpurun_out/ab_doom9_c3.txt; exit 1; }
cat gpurun_out/ab_doom9_c3.txt
timeout -k 10 300 python -u tools/abtime.py --config C3 --scene s_glass --flags 48 --rounds 11 --frames 20 head=$L hard=ab/doom_hard.so > gpurun_out/ab_doom9_glass.txt 2>&1 || { echo "glass ab failed"; tail -20 gpurun_out/ab_doom9_glass.txt; exit 1; }
cat gpurun_out/ab_doom9_glass.txt
