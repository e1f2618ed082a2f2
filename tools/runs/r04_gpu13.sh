#!/bin/bash
# round 4: block order with the LDS sort -- the sort launch alone (order not
# used), heavy-first 512 / 2048, full longest-first, row-major; C5
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/../.." && pwd)}"
cd "$ROOT"; mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_block_order_gpu.py -x -q --timeout 120 --timeout-method thread > gpurun_out/t_order.log 2>&1 || { echo "test failed"; tail -30 gpurun_out/t_order.log; exit 1; }
tail -1 gpurun_out/t_order.log
timeout -k 10 500 python tools/abtime.py --config C5 --flags 48 --rounds 5 --frames 10 noorder=ab/lean_head4_noorder.so sortonly=ab/lean_head5_sortonly.so h512=ab/lean_head5_h512.so h2k=ab/lean_head5.so lpt=ab/lean_head5_lpt.so > gpurun_out/ab_order3_c5.txt 2>&1 || { echo "ab failed"; tail gpurun_out/ab_order3_c5.txt; exit 1; }
cat gpurun_out/ab_order3_c5.txt
