#!/bin/bash
# round 6: the soft-shadow unit (EXT 2) with the max-ilp schedule (ab/e2ilp.so) against the head on C5
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/../.." && pwd)}"
cd "$ROOT"; mkdir -p gpurun_out
L=voxmap_amd/libvoxmap_hip.so
timeout -k 10 500 python -u tools/abtime.py --config C5 --flags 48 --rounds 7 --frames 10 head=$L e2ilp=ab/e2ilp.so > gpurun_out/ab_e2ilp_c5.txt 2>&1 || { echo "c5 ab failed"; tail -20 gpurun_out/ab_e2ilp_c5.txt; exit 1; }
cat gpurun_out/ab_e2ilp_c5.txt
