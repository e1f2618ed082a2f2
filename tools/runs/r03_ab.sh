#!/bin/bash
# round 3 A/B helper: a parity subset of the GPU tests on the current build, then
# interleaved timings of ab/lib_base.so (the committed head) against it.
# usage (on the box): bash tools/runs/r03_ab.sh [pytest -k expression]
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/../.." && pwd)}"
cd "$ROOT"; mkdir -p gpurun_out
K="${1:-small_frames or baseline_sizes_full_frame or extensions_baseline_full_frame or campus or edge_params or ragged or extensions_bit_exact}"
timeout -k 10 600 python -u -m pytest tests/test_parity_gpu.py tests/test_golden.py -m gpu -x -q --timeout 300 --timeout-method thread -k "$K" > gpurun_out/pytest_ab.log 2>&1
rc=$?; tail -4 gpurun_out/pytest_ab.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python tools/abtime.py --config C3 --flags 0,48 --rounds 9 base=ab/lib_base.so $AB_EXTRA new=voxmap_amd/libvoxmap_hip.so > gpurun_out/ab_c3.txt 2>&1 || { echo "ab c3 failed"; tail gpurun_out/ab_c3.txt; exit 1; }
cat gpurun_out/ab_c3.txt
if [ -n "$AB_C5" ]; then
timeout -k 10 300 python tools/abtime.py --config C5 --flags 48 --rounds 5 --frames 10 base=ab/lib_base.so new=voxmap_amd/libvoxmap_hip.so > gpurun_out/ab_c5.txt 2>&1 || { echo "ab c5 failed"; tail gpurun_out/ab_c5.txt; exit 1; }
cat gpurun_out/ab_c5.txt
fi
