#!/bin/bash
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/../.." && pwd)}"
cd "$ROOT"; mkdir -p gpurun_out
timeout -k 10 120 tools/micro/sqrt_ranged_check > gpurun_out/sqrt_ranged_check.txt 2>&1; rc=$?; cat gpurun_out/sqrt_ranged_check.txt; [ $rc -eq 0 ] || exit $rc
AB_EXTRA="a=ab/lib_a.so b=ab/lib_b.so" bash tools/runs/r03_ab.sh
