#!/bin/bash
# round 6: doom codes carrying h only (hmax from MAX and the cone window, the
# texel read from the plain channel when a march goes on) against the first
# form (h <= 13, texel <= 8 in the code: ab/doom13.so) and the pre-doom head
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/../.." && pwd)}"
cd "$ROOT"; mkdir -p gpurun_out
L=voxmap_amd/libvoxmap_hip.so
timeout -k 10 400 python -u -m pytest tests/test_doom_gpu.py tests/test_exit_gpu.py -x -q --timeout 200 --timeout-method thread > gpurun_out/doom4_tests.log 2>&1 || { echo "doom tests failed"; tail -30 gpurun_out/doom4_tests.log; exit 1; }
tail -1 gpurun_out/doom4_tests.log
timeout -k 10 300 python -u -m pytest tests/test_parity_gpu.py -x -q -k "soft_pool" --timeout 200 --timeout-method thread > gpurun_out/doom4_pool.log 2>&1 || { echo "pool test failed"; tail -30 gpurun_out/doom4_pool.log; exit 1; }
tail -1 gpurun_out/doom4_pool.log
timeout -k 10 500 python -u tools/abtime.py --config C5 --flags 48 --rounds 7 --frames 10 pre=ab/pre_doom.so doom13=ab/doom13.so head=$L nodoom=$L+131072 > gpurun_out/ab_doom4_c5.txt 2>&1 || { echo "c5 ab failed"; tail -20 gpurun_out/ab_doom4_c5.txt; exit 1; }
cat gpurun_out/ab_doom4_c5.txt
timeout -k 10 300 python -u tools/doom_build_time.py --out gpurun_out/doom_build.json > gpurun_out/doom_build.log 2>&1 || { echo "build time failed"; tail -20 gpurun_out/doom_build.log; exit 1; }
cat gpurun_out/doom_build.log
