#!/bin/bash
# round 4: the quad-relative split's cost -- per-step speculative quad-offset
# loads (QSPEC, product) against the end-of-walk table read (ab/lib_noqspec.so),
# each against its own unit-cell split (0x800); then the quad/exit GPU tests.
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/../.." && pwd)}"
cd "$ROOT"; mkdir -p gpurun_out
timeout -k 10 400 python tools/abtime.py --config C3 --flags 48,2096,0,2048 --rounds 7 new=voxmap_amd/libvoxmap_hip.so endload=ab/lib_noqspec.so > gpurun_out/ab_qspec_c3.txt 2>&1 || { echo "ab c3 failed"; tail gpurun_out/ab_qspec_c3.txt; exit 1; }
cat gpurun_out/ab_qspec_c3.txt
timeout -k 10 400 python tools/abtime.py --config C5 --flags 48,2096 --rounds 3 --frames 10 new=voxmap_amd/libvoxmap_hip.so endload=ab/lib_noqspec.so > gpurun_out/ab_qspec_c5.txt 2>&1 || { echo "ab c5 failed"; tail gpurun_out/ab_qspec_c5.txt; exit 1; }
cat gpurun_out/ab_qspec_c5.txt
timeout -k 10 600 python -u -m pytest tests/test_quad_gpu.py tests/test_exit_gpu.py -x -q --timeout 300 --timeout-method thread > gpurun_out/pytest_quad_b.log 2>&1
rc=$?; tail -3 gpurun_out/pytest_quad_b.log; exit $rc
