#!/bin/bash
# round 6: doom codes carrying the crossing bound C(h) (head; hmax from
# 1 + 2 C(h) < MAX) against codes carrying h with the (h + 1) 2 (kx + ky + 1)
# landing bound (ab/doom_q8_v1.so): GPU doom + exit tests, C5 A/B, build time
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/../.." && pwd)}"
cd "$ROOT"; mkdir -p gpurun_out
L=voxmap_amd/libvoxmap_hip.so
timeout -k 10 400 python -u -m pytest tests/test_doom_gpu.py tests/test_exit_gpu.py -x -q --timeout 200 --timeout-method thread > gpurun_out/doom7_tests.log 2>&1 || { echo "doom tests failed"; tail -30 gpurun_out/doom7_tests.log; exit 1; }
tail -1 gpurun_out/doom7_tests.log
timeout -k 10 500 python -u tools/abtime.py --config C5 --flags 48 --rounds 7 --frames 10 pre=ab/pre_doom.so hbound=ab/doom_q8_v1.so cbound=$L > gpurun_out/ab_doom7_c5.txt 2>&1 || { echo "c5 ab failed"; tail -20 gpurun_out/ab_doom7_c5.txt; exit 1; }
cat gpurun_out/ab_doom7_c5.txt
timeout -k 10 300 python -u tools/doom_build_time.py --out gpurun_out/doom_build_c.json > gpurun_out/doom_build_c.log 2>&1 || { echo "build time failed"; tail -20 gpurun_out/doom_build_c.log; exit 1; }
tail -1 gpurun_out/doom_build_c.log
