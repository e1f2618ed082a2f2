#!/bin/bash
# round 6: the doom table's hmax with a landing margin (codes only where the stop
# rule holds up to landing 1 + M: fewer late codes) -- M = 0 (head), 8, 20
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/../.." && pwd)}"
cd "$ROOT"; mkdir -p gpurun_out
L=voxmap_amd/libvoxmap_hip.so
timeout -k 10 400 python -u tools/abtime.py --config C3 --flags 48,0 --rounds 11 --frames 20 head=$L m8=ab/margin8.so m20=ab/margin20.so > gpurun_out/ab_margin_c3.txt 2>&1 || { echo "c3 ab failed"; tail -20 gpurun_out/ab_margin_c3.txt; exit 1; }
cat gpurun_out/ab_margin_c3.txt
timeout -k 10 400 python -u tools/abtime.py --config C5 --flags 48 --rounds 5 --frames 10 head=$L m8=ab/margin8.so m20=ab/margin20.so > gpurun_out/ab_margin_c5.txt 2>&1 || { echo "c5 ab failed"; tail -20 gpurun_out/ab_margin_c5.txt; exit 1; }
cat gpurun_out/ab_margin_c5.txt
