#!/bin/bash
# round 6 A/B 1: block-row rotation (rows from 33 % / 55 % down, wrapping) and a
# wave-uniform tie branch in the march loop, against the head: C5 and C3
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/../.." && pwd)}"
cd "$ROOT"; mkdir -p gpurun_out
V="head=voxmap_amd/libvoxmap_hip.so rot33=ab/rot33.so rot55=ab/rot55.so tieb=ab/tieb.so"
timeout -k 10 500 python -u tools/abtime.py --config C5 --flags 48 --rounds 5 --frames 10 $V > gpurun_out/ab1_c5.txt 2>&1 || { echo "c5 ab failed"; tail -20 gpurun_out/ab1_c5.txt; exit 1; }
cat gpurun_out/ab1_c5.txt
timeout -k 10 300 python -u tools/abtime.py --config C3 --flags 48,0 --rounds 7 --frames 20 $V > gpurun_out/ab1_c3.txt 2>&1 || { echo "c3 ab failed"; tail -20 gpurun_out/ab1_c3.txt; exit 1; }
cat gpurun_out/ab1_c3.txt
