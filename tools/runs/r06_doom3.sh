#!/bin/bash
# round 6: where the soft march resolves a doom code -- after its loop with a
# per-lane landing count (head) or inside the loop at the wave's landing
# (ab/doom_inloop.so) -- against the pre-doom head, on C5 and S-glass soft
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/../.." && pwd)}"
cd "$ROOT"; mkdir -p gpurun_out
L=voxmap_amd/libvoxmap_hip.so
timeout -k 10 300 python -u -m pytest tests/test_doom_gpu.py -x -q --timeout 200 --timeout-method thread > gpurun_out/doom3_tests.log 2>&1 || { echo "doom tests failed"; tail -30 gpurun_out/doom3_tests.log; exit 1; }
tail -1 gpurun_out/doom3_tests.log
timeout -k 10 500 python -u tools/abtime.py --config C5 --flags 48 --rounds 7 --frames 10 pre=ab/pre_doom.so post=$L inloop=ab/doom_inloop.so nodoom=$L+131072 > gpurun_out/ab_doom3_c5.txt 2>&1 || { echo "c5 ab failed"; tail -20 gpurun_out/ab_doom3_c5.txt; exit 1; }
cat gpurun_out/ab_doom3_c5.txt
timeout -k 10 300 python -u tools/abtime.py --config C5 --scene s_proc --flags 48 --rounds 7 --frames 10 pre=ab/pre_doom.so post=$L inloop=ab/doom_inloop.so > gpurun_out/ab_doom3_c5proc.txt 2>&1 || { echo "c5proc ab failed"; tail -20 gpurun_out/ab_doom3_c5proc.txt; exit 1; }
cat gpurun_out/ab_doom3_c5proc.txt
