#!/bin/bash
# round 4: the per-render cone reader event (head2) against none on a
# single-stream scene (head3), no quad split (noquad3) and r03; then C5
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/../.." && pwd)}"
cd "$ROOT"; mkdir -p gpurun_out
timeout -k 10 500 python tools/abtime.py --config C3 --flags 0,48 --rounds 9 r03=ab/lib_r03.so head2=ab/lean_head2.so head3=ab/lean_head3.so noquad3=ab/lean_noquad3.so nosky2=ab/lean_nosky2.so > gpurun_out/ab_event.txt 2>&1 || { echo "ab failed"; tail gpurun_out/ab_event.txt; exit 1; }
cat gpurun_out/ab_event.txt
timeout -k 10 500 python tools/abtime.py --config C5 --flags 48 --rounds 3 --frames 10 r03=ab/lib_r03.so head3=ab/lean_head3.so noquad3=ab/lean_noquad3.so > gpurun_out/ab_event_c5.txt 2>&1 || { echo "ab failed"; tail gpurun_out/ab_event_c5.txt; exit 1; }
cat gpurun_out/ab_event_c5.txt
