#!/bin/bash
# round 4: adaptive block order (longest blocks of the last frame first) on C5
# and C3 against row-major (noorder) and r03
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/../.." && pwd)}"
cd "$ROOT"; mkdir -p gpurun_out
timeout -k 10 500 python tools/abtime.py --config C5 --flags 48 --rounds 5 --frames 10 r03=ab/lib_r03.so noorder=ab/lean_head4_noorder.so order=ab/lean_head4.so > gpurun_out/ab_order_c5.txt 2>&1 || { echo "ab failed"; tail gpurun_out/ab_order_c5.txt; exit 1; }
cat gpurun_out/ab_order_c5.txt
timeout -k 10 500 python tools/abtime.py --config C3 --flags 0,48 --rounds 7 r03=ab/lib_r03.so noorder=ab/lean_head4_noorder.so allorder=ab/lean_head4_allorder.so head3=ab/lean_head3.so > gpurun_out/ab_order_c3.txt 2>&1 || { echo "ab failed"; tail gpurun_out/ab_order_c3.txt; exit 1; }
cat gpurun_out/ab_order_c3.txt
