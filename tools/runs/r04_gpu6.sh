#!/bin/bash
# round 4: what the head's v1 frame pays against the round-3 head -- A/A (r03 twice),
# the quad split, the sky noise skip, the qcopy allocation (lean A/B builds)
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/../.." && pwd)}"
cd "$ROOT"; mkdir -p gpurun_out
timeout -k 10 500 python tools/abtime.py --config C3 --flags 0,48 --rounds 9 r03=ab/lib_r03.so r03b=ab/lib_r03b.so noquad=ab/lean_noquad.so nosky=ab/lean_nosky.so head=ab/lean_head.so headoldsky=ab/lean_headoldsky.so > gpurun_out/ab_v1_bisect.txt 2>&1 || { echo "ab failed"; tail gpurun_out/ab_v1_bisect.txt; exit 1; }
cat gpurun_out/ab_v1_bisect.txt
