#!/bin/bash
# round 4: does the order in which abtime creates the variants' scenes (their
# device addresses) move the timings?  The same libraries, another order.
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/../.." && pwd)}"
cd "$ROOT"; mkdir -p gpurun_out
timeout -k 10 500 python tools/abtime.py --config C3 --flags 0,48 --rounds 9 nosky=ab/lean_nosky.so r03=ab/lib_r03.so head=ab/lean_head.so r03b=ab/lib_r03b.so > gpurun_out/ab_order.txt 2>&1 || { echo "ab failed"; tail gpurun_out/ab_order.txt; exit 1; }
cat gpurun_out/ab_order.txt
timeout -k 10 500 python tools/abtime.py --config C3 --flags 0,48 --rounds 9 head=ab/lean_head.so > gpurun_out/ab_alone_head.txt 2>&1 && cat gpurun_out/ab_alone_head.txt
timeout -k 10 500 python tools/abtime.py --config C3 --flags 0,48 --rounds 9 r03=ab/lib_r03.so > gpurun_out/ab_alone_r03.txt 2>&1 && cat gpurun_out/ab_alone_r03.txt
