#!/bin/bash
# round 4: G-buffer cells as exact fp32 (no int <-> float converts in the
# consumers) -- GPU suite, then A/B against the same sources before the change
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/../.." && pwd)}"
cd "$ROOT"; mkdir -p gpurun_out
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/gpu_tests_r04c.log 2>&1 || { echo "gpu tests failed rc=$?"; grep -E "FAILED|Error|passed|failed" gpurun_out/gpu_tests_r04c.log | tail -20; exit 1; }
tail -2 gpurun_out/gpu_tests_r04c.log
timeout -k 10 500 python tools/abtime.py --config C3 --flags 0,48 --rounds 9 pre=ab/lean_pre.so post=ab/lean_post.so > gpurun_out/ab_fcell_c3.txt 2>&1 || { echo "ab failed"; tail gpurun_out/ab_fcell_c3.txt; exit 1; }
cat gpurun_out/ab_fcell_c3.txt
timeout -k 10 500 python tools/abtime.py --config C5 --flags 48 --rounds 3 --frames 10 pre=ab/lean_pre.so post=ab/lean_post.so > gpurun_out/ab_fcell_c5.txt 2>&1 || { echo "ab failed"; tail gpurun_out/ab_fcell_c5.txt; exit 1; }
cat gpurun_out/ab_fcell_c5.txt
