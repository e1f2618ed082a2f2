#!/bin/bash
# round 6: the doom table on 8 x 8 sub-cells per cell (head) against 4 x 4
# (ab/doom_q4.so): GPU doom tests, interleaved C5 A/B, build time
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/../.." && pwd)}"
cd "$ROOT"; mkdir -p gpurun_out
L=voxmap_amd/libvoxmap_hip.so
timeout -k 10 400 python -u -m pytest tests/test_doom_gpu.py -x -q --timeout 200 --timeout-method thread > gpurun_out/doom5_tests.log 2>&1 || { echo "doom tests failed"; tail -30 gpurun_out/doom5_tests.log; exit 1; }
tail -1 gpurun_out/doom5_tests.log
timeout -k 10 500 python -u tools/abtime.py --config C5 --flags 48 --rounds 7 --frames 10 pre=ab/pre_doom.so q4=ab/doom_q4.so q8=$L > gpurun_out/ab_doom5_c5.txt 2>&1 || { echo "c5 ab failed"; tail -20 gpurun_out/ab_doom5_c5.txt; exit 1; }
cat gpurun_out/ab_doom5_c5.txt
timeout -k 10 300 python -u tools/doom_build_time.py --out gpurun_out/doom_build_q8.json > gpurun_out/doom_build_q8.log 2>&1 || { echo "build time failed"; tail -20 gpurun_out/doom_build_q8.log; exit 1; }
cat gpurun_out/doom_build_q8.log
