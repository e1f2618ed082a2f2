#!/bin/bash
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/../.." && pwd)}"
cd "$ROOT"; mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_parity_gpu.py -m gpu -x -q --timeout 300 --timeout-method thread -k "small_frames or baseline_sizes_full_frame or extensions_baseline_full_frame or extensions_bit_exact" > gpurun_out/pytest_ab.log 2>&1
rc=$?; tail -3 gpurun_out/pytest_ab.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python tools/abtime.py --config C3 --flags 0,48 --rounds 11 a=ab/lib_a.so new=voxmap_amd/libvoxmap_hip.so > gpurun_out/ab_c3.txt 2>&1 || { echo "ab failed"; tail gpurun_out/ab_c3.txt; exit 1; }
cat gpurun_out/ab_c3.txt
timeout -k 10 300 python tools/abtime.py --config C3 --flags 48,0,8,1,2,4,16,32,49,50,52 --rounds 5 new=voxmap_amd/libvoxmap_hip.so > gpurun_out/phases_c3.txt 2>&1 || { echo "phases failed"; tail gpurun_out/phases_c3.txt; exit 1; }
cat gpurun_out/phases_c3.txt
