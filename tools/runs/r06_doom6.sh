#!/bin/bash
# round 6: the doom layer kernel without integer division (head) against the
# first 8 x 8 sub-cell build (ab/doom_q8_v1.so): GPU doom tests, build time, C5 frames (v2: unrolled staging)
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/../.." && pwd)}"
cd "$ROOT"; mkdir -p gpurun_out
L=voxmap_amd/libvoxmap_hip.so
timeout -k 10 400 python -u -m pytest tests/test_doom_gpu.py tests/test_exit_gpu.py -x -q --timeout 200 --timeout-method thread > gpurun_out/doom6_tests.log 2>&1 || { echo "doom tests failed"; tail -30 gpurun_out/doom6_tests.log; exit 1; }
tail -1 gpurun_out/doom6_tests.log
timeout -k 10 300 python -u tools/doom_build_time.py --out gpurun_out/doom_build_v2.json > gpurun_out/doom_build_v2.log 2>&1 || { echo "build time failed"; tail -20 gpurun_out/doom_build_v2.log; exit 1; }
cat gpurun_out/doom_build_v2.log
timeout -k 10 300 python -u tools/abtime.py --config C5 --flags 48 --rounds 3 --frames 10 v1=ab/doom_q8_v1.so head=$L > gpurun_out/ab_doom6_c5.txt 2>&1 || { echo "c5 ab failed"; tail -20 gpurun_out/ab_doom6_c5.txt; exit 1; }
cat gpurun_out/ab_doom6_c5.txt
