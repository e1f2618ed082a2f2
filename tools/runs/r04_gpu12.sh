#!/bin/bash
# round 4: block order -- heavy-first (VX_ORDER_HEAVY 512 / 2048 / 8192 blocks),
# the rest row-major, against row-major and r03; GPU test of identical frames
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/../.." && pwd)}"
cd "$ROOT"; mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_block_order_gpu.py -x -q --timeout 120 --timeout-method thread > gpurun_out/t_order.log 2>&1 || { echo "test failed"; tail -30 gpurun_out/t_order.log; exit 1; }
tail -2 gpurun_out/t_order.log
timeout -k 10 500 python tools/abtime.py --config C5 --flags 48 --rounds 5 --frames 10 r03=ab/lib_r03.so noorder=ab/lean_head4_noorder.so h512=ab/lean_head5_h512.so h2k=ab/lean_head5.so h8k=ab/lean_head5_h8k.so > gpurun_out/ab_order2_c5.txt 2>&1 || { echo "ab failed"; tail gpurun_out/ab_order2_c5.txt; exit 1; }
cat gpurun_out/ab_order2_c5.txt
timeout -k 10 500 python tools/abtime.py --config C3 --flags 0,48 --rounds 7 noorder=ab/lean_head4_noorder.so all2k=ab/lean_head5_all.so > gpurun_out/ab_order2_c3.txt 2>&1 || { echo "ab failed"; tail gpurun_out/ab_order2_c3.txt; exit 1; }
cat gpurun_out/ab_order2_c3.txt
