#!/bin/bash
# round 6: the hard shadow's doom codes resolved inside the march loop (head,
# kDoomIn) against resolved after it (ab/doom_hard.so, kDoomAfter; spills in
# the hard units' step loop), and the head without the table (VX_FLAG_NO_DOOM):
# C3 full quality, v1, REFLECT_ALL, S-glass; C5 (soft: kDoomAfter in both)
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/../.." && pwd)}"
cd "$ROOT"; mkdir -p gpurun_out
L=voxmap_amd/libvoxmap_hip.so
timeout -k 10 400 python -u tools/abtime.py --config C3 --flags 48,0,8240 --rounds 11 --frames 20 inloop=$L after=ab/doom_hard.so nodoom=$L+131072 > gpurun_out/ab_doom10_c3.txt 2>&1 || { echo "c3 ab failed"; tail -20 gpurun_out/ab_doom10_c3.txt; exit 1; }
cat gpurun_out/ab_doom10_c3.txt
timeout -k 10 300 python -u tools/abtime.py --config C3 --scene s_glass --flags 48 --rounds 11 --frames 20 inloop=$L after=ab/doom_hard.so nodoom=$L+131072 > gpurun_out/ab_doom10_glass.txt 2>&1 || { echo "glass ab failed"; tail -20 gpurun_out/ab_doom10_glass.txt; exit 1; }
cat gpurun_out/ab_doom10_glass.txt
timeout -k 10 400 python -u tools/abtime.py --config C5 --flags 48 --rounds 5 --frames 10 inloop=$L after=ab/doom_hard.so > gpurun_out/ab_doom10_c5.txt 2>&1 || { echo "c5 ab failed"; tail -20 gpurun_out/ab_doom10_c5.txt; exit 1; }
cat gpurun_out/ab_doom10_c5.txt
