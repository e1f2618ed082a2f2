#!/bin/bash
# round 6: the sun doom table -- its GPU tests (+ the exit-table suite), the
# cone copy's build time with and without it, and an interleaved A/B of the
# default (doom) against VX_FLAG_NO_DOOM on C3 (full, v1) and C5
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/../.." && pwd)}"
cd "$ROOT"; mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_doom_gpu.py tests/test_exit_gpu.py -x -v --timeout 300 --timeout-method thread > gpurun_out/doom_tests.log 2>&1 || { echo "doom tests failed rc=$?"; grep -E "FAILED|Error|assert|passed|failed" gpurun_out/doom_tests.log | tail -30; exit 1; }
tail -2 gpurun_out/doom_tests.log
timeout -k 10 300 python -u tools/doom_build_time.py --out gpurun_out/doom_build.json > gpurun_out/doom_build.log 2>&1 || { echo "build time failed"; tail -20 gpurun_out/doom_build.log; exit 1; }
cat gpurun_out/doom_build.log
timeout -k 10 300 python -u tools/abtime.py --config C3 --flags 48,0 --rounds 9 --frames 20 doom=voxmap_amd/libvoxmap_hip.so nodoom=voxmap_amd/libvoxmap_hip.so+131072 > gpurun_out/ab_doom_c3.txt 2>&1 || { echo "c3 ab failed"; tail -20 gpurun_out/ab_doom_c3.txt; exit 1; }
cat gpurun_out/ab_doom_c3.txt
timeout -k 10 400 python -u tools/abtime.py --config C5 --flags 48 --rounds 5 --frames 10 doom=voxmap_amd/libvoxmap_hip.so nodoom=voxmap_amd/libvoxmap_hip.so+131072 > gpurun_out/ab_doom_c5.txt 2>&1 || { echo "c5 ab failed"; tail -20 gpurun_out/ab_doom_c5.txt; exit 1; }
cat gpurun_out/ab_doom_c5.txt
