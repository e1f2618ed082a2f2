#!/bin/bash
# round 4: the face table allocated after the per-step arrays (nosky2, head2)
# against the same code with it allocated before them (nosky, head) and r03
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/../.." && pwd)}"
cd "$ROOT"; mkdir -p gpurun_out
timeout -k 10 500 python tools/abtime.py --config C3 --flags 0,48 --rounds 9 r03=ab/lib_r03.so nosky=ab/lean_nosky.so nosky2=ab/lean_nosky2.so head=ab/lean_head.so head2=ab/lean_head2.so > gpurun_out/ab_alloc_order.txt 2>&1 || { echo "ab failed"; tail gpurun_out/ab_alloc_order.txt; exit 1; }
cat gpurun_out/ab_alloc_order.txt
timeout -k 10 500 python tools/abtime.py --config C5 --flags 48 --rounds 3 --frames 10 r03=ab/lib_r03.so head2=ab/lean_head2.so > gpurun_out/ab_alloc_order_c5.txt 2>&1 || { echo "ab failed"; tail gpurun_out/ab_alloc_order_c5.txt; exit 1; }
cat gpurun_out/ab_alloc_order_c5.txt
