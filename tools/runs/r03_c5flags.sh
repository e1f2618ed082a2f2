#!/bin/bash
# round 3: C5 with the sun exit tables -- default per-sample loop vs the pooled wave pass (VX_FLAG_SOFT_POOL)
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/../.." && pwd)}"
cd "$ROOT"; mkdir -p gpurun_out
timeout -k 10 300 python tools/abtime.py --config C5 --flags 48,176 --rounds 5 --frames 10 new=voxmap_amd/libvoxmap_hip.so > gpurun_out/c5_pool.txt 2>&1 || { echo "c5 pool failed"; tail gpurun_out/c5_pool.txt; exit 1; }
cat gpurun_out/c5_pool.txt
