#!/bin/bash
# round 4: quad-relative G-buffer -- smoke, the new GPU tests, every GPU test,
# then the in-process A/B of the split (flags 0x800 = VX_FLAG_UNIT_GBUF).
# Each GPU step has its own time limit; the first failure ends the script.
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/../.." && pwd)}"
cd "$ROOT"; mkdir -p gpurun_out
timeout -k 10 180 python -c 'import __graft_entry__ as g; g.smoke()' > gpurun_out/smoke.log 2>&1 || { echo "smoke failed rc=$?"; tail -20 gpurun_out/smoke.log; exit 1; }
tail -2 gpurun_out/smoke.log
timeout -k 10 600 python -u -m pytest tests/test_quad_gpu.py -x -v --timeout 300 --timeout-method thread > gpurun_out/pytest_quad.log 2>&1
rc=$?; tail -5 gpurun_out/pytest_quad.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python tools/abtime.py --config C3 --flags 48,2096,0,2048 --rounds 7 new=voxmap_amd/libvoxmap_hip.so > gpurun_out/ab_quad_c3.txt 2>&1 || { echo "ab c3 failed"; tail gpurun_out/ab_quad_c3.txt; exit 1; }
cat gpurun_out/ab_quad_c3.txt
timeout -k 10 300 python tools/abtime.py --config C5 --flags 48,2096 --rounds 3 --frames 10 new=voxmap_amd/libvoxmap_hip.so > gpurun_out/ab_quad_c5.txt 2>&1 || { echo "ab c5 failed"; tail gpurun_out/ab_quad_c5.txt; exit 1; }
cat gpurun_out/ab_quad_c5.txt
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1
rc=$?; tail -5 gpurun_out/pytest_gpu.log; exit $rc
