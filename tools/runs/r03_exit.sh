#!/bin/bash
# round 3: sun exit tables -- identical frames with the cone + orthant tables,
# the orthant tables only and none (and the fetch counts), every GPU test, then
# interleaved timings against the build without them (ab/lib_base.so)
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/../.." && pwd)}"
cd "$ROOT"; mkdir -p gpurun_out
timeout -k 10 180 python tools/exit_probe.py --config C3 --flags 0,48 > gpurun_out/exit_c3.txt 2>&1 || { echo "probe c3 failed"; tail gpurun_out/exit_c3.txt; exit 1; }
cat gpurun_out/exit_c3.txt
timeout -k 10 240 python tools/exit_probe.py --config C5 --flags 48 --frames 5 > gpurun_out/exit_c5.txt 2>&1 || { echo "probe c5 failed"; tail gpurun_out/exit_c5.txt; exit 1; }
cat gpurun_out/exit_c5.txt
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1
rc=$?; tail -5 gpurun_out/pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python tools/abtime.py --config C3 --flags 0,48 --rounds 9 base=ab/lib_base.so new=voxmap_amd/libvoxmap_hip.so > gpurun_out/ab_c3.txt 2>&1 || { echo "ab c3 failed"; tail gpurun_out/ab_c3.txt; exit 1; }
cat gpurun_out/ab_c3.txt
timeout -k 10 300 python tools/abtime.py --config C5 --flags 48 --rounds 5 --frames 10 base=ab/lib_base.so new=voxmap_amd/libvoxmap_hip.so > gpurun_out/ab_c5.txt 2>&1 || { echo "ab c5 failed"; tail gpurun_out/ab_c5.txt; exit 1; }
cat gpurun_out/ab_c5.txt
