#!/bin/bash
# round 6: the doom build with unrolled window maxima (head) against the
# previous build (ab/doom_build_v2.so): GPU doom tests, build time, C5 frames
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/../.." && pwd)}"
cd "$ROOT"; mkdir -p gpurun_out
L=voxmap_amd/libvoxmap_hip.so
timeout -k 10 400 python -u -m pytest tests/test_doom_gpu.py tests/test_exit_gpu.py -x -q --timeout 200 --timeout-method thread > gpurun_out/doom11_tests.log 2>&1 || { echo "doom tests failed"; tail -30 gpurun_out/doom11_tests.log; exit 1; }
tail -1 gpurun_out/doom11_tests.log
timeout -k 10 300 python -u tools/doom_build_time.py --out gpurun_out/doom_build_v3.json > gpurun_out/doom_build_v3.log 2>&1 || { echo "build time failed"; tail -20 gpurun_out/doom_build_v3.log; exit 1; }
cat gpurun_out/doom_build_v3.log
timeout -k 10 300 python -u tools/abtime.py --config C5 --flags 48 --rounds 3 --frames 10 prev=ab/doom_build_v2.so head=$L > gpurun_out/ab_doom11_c5.txt 2>&1 || { echo "c5 ab failed"; tail -20 gpurun_out/ab_doom11_c5.txt; exit 1; }
cat gpurun_out/ab_doom11_c5.txt
