#!/bin/bash
# round 4: the tile entry box -- frames against the oracle, then A/B timing
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/../.." && pwd)}"
cd "$ROOT"; mkdir -p gpurun_out
timeout -k 10 400 python -u tools/tile_box_check.py > gpurun_out/tile_box_check.txt 2>&1; echo "check rc=$?"; cat gpurun_out/tile_box_check.txt | grep -v amdgpu
timeout -k 10 500 python tools/abtime.py --config C3 --flags 0,48,8 --rounds 7 notb=ab/lean_notb.so tb=ab/lean_tb.so > gpurun_out/ab_tb_c3.txt 2>&1 || { echo "ab failed"; tail gpurun_out/ab_tb_c3.txt; exit 1; }
cat gpurun_out/ab_tb_c3.txt
timeout -k 10 500 python tools/abtime.py --config C5 --flags 48 --rounds 3 --frames 10 notb=ab/lean_notb.so tb=ab/lean_tb.so > gpurun_out/ab_tb_c5.txt 2>&1 || { echo "ab failed"; tail gpurun_out/ab_tb_c5.txt; exit 1; }
cat gpurun_out/ab_tb_c5.txt
