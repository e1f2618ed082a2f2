#!/bin/bash
# round 3: every GPU test on the current build, then A/B against ab/lib_base.so (C3 v1 + full, C5)
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/../.." && pwd)}"
cd "$ROOT"; mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1
rc=$?; tail -4 gpurun_out/pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
bash tools/runs/r03_ab2.sh new=voxmap_amd/libvoxmap_hip.so
