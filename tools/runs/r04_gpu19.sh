#!/bin/bash
# round 4: EXT 5/6 (glass in draw order, REFLECT_ALL) in their own kernel with
# a register budget of their own -- 6 waves/SIMD (head), 7, and the 8-wave
# 80-SGPR budget of the other kernels; GPU suite on the head first
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/../.." && pwd)}"
cd "$ROOT"; mkdir -p gpurun_out
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/gpu_tests_r04d.log 2>&1 || { echo "gpu tests failed rc=$?"; grep -E "FAILED|Error|passed|failed" gpurun_out/gpu_tests_r04d.log | tail -20; exit 1; }
tail -2 gpurun_out/gpu_tests_r04d.log
timeout -k 10 600 python tools/abtime.py --config C3 --flags 8240,4144,48 --rounds 5 --frames 10 gen6=voxmap_amd/libvoxmap_hip.so gen7=ab/full_gen7.so gen8=ab/full_gen8.so > gpurun_out/ab_gen_c3.txt 2>&1 || { echo "ab failed"; tail gpurun_out/ab_gen_c3.txt; exit 1; }
cat gpurun_out/ab_gen_c3.txt
