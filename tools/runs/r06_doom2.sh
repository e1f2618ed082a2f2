#!/bin/bash
# round 6: the doom table against the round's previous head (ab/pre_doom.so):
# interleaved A/B on C3 (full, v1), S-glass C3 and C5; then the whole GPU suite and smoke()
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/../.." && pwd)}"
cd "$ROOT"; mkdir -p gpurun_out
L=voxmap_amd/libvoxmap_hip.so
timeout -k 10 300 python -u tools/abtime.py --config C3 --flags 48,0 --rounds 9 --frames 20 pre=ab/pre_doom.so doom=$L nodoom=$L+131072 > gpurun_out/ab_doom2_c3.txt 2>&1 || { echo "c3 ab failed"; tail -20 gpurun_out/ab_doom2_c3.txt; exit 1; }
cat gpurun_out/ab_doom2_c3.txt
timeout -k 10 300 python -u tools/abtime.py --config C3 --scene s_glass --flags 48 --rounds 9 --frames 20 pre=ab/pre_doom.so doom=$L nodoom=$L+131072 > gpurun_out/ab_doom2_glass.txt 2>&1 || { echo "glass ab failed"; tail -20 gpurun_out/ab_doom2_glass.txt; exit 1; }
cat gpurun_out/ab_doom2_glass.txt
timeout -k 10 400 python -u tools/abtime.py --config C5 --flags 48 --rounds 5 --frames 10 pre=ab/pre_doom.so doom=$L nodoom=$L+131072 > gpurun_out/ab_doom2_c5.txt 2>&1 || { echo "c5 ab failed"; tail -20 gpurun_out/ab_doom2_c5.txt; exit 1; }
cat gpurun_out/ab_doom2_c5.txt
TAG=r06_doom bash tools/runs/r06_gpu_tests.sh
