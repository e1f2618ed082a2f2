#!/bin/bash
# round 3, GPU call 2: TA micro (scattered lines), GPU tests of the cleaned kernel, A/B vs the r02 head
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/../.." && pwd)}"
cd "$ROOT"; mkdir -p gpurun_out
timeout -k 10 120 tools/micro/ta_rate > gpurun_out/ta_rate2.txt 2>&1 || { echo "ta_rate failed"; exit 1; }
cat gpurun_out/ta_rate2.txt
timeout -k 10 180 python -c 'import __graft_entry__ as g; g.smoke()' > gpurun_out/smoke.log 2>&1 || { echo "smoke failed rc=$?"; tail -20 gpurun_out/smoke.log; exit 1; }
tail -2 gpurun_out/smoke.log
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1
rc=$?; tail -5 gpurun_out/pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 240 python tools/abtime.py --config C3 --flags 0,48 --rounds 7 old=ab/lib_r02head.so new=voxmap_amd/libvoxmap_hip.so > gpurun_out/ab_c3.txt 2>&1 || { echo "ab c3 failed"; tail gpurun_out/ab_c3.txt; exit 1; }
cat gpurun_out/ab_c3.txt
timeout -k 10 300 python tools/abtime.py --config C5 --flags 48 --rounds 5 --frames 10 old=ab/lib_r02head.so new=voxmap_amd/libvoxmap_hip.so > gpurun_out/ab_c5.txt 2>&1 || { echo "ab c5 failed"; tail gpurun_out/ab_c5.txt; exit 1; }
cat gpurun_out/ab_c5.txt
