#!/bin/bash
# round 6: the one-GPU multi-rank rehearsal (bench.py --gpus 2 --gather gloo) and the
# glass-lattice timing (non-STATS launches, event-timed)
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/../.." && pwd)}"
cd "$ROOT"; mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_mgpu_rehearsal_gpu.py -m gpu -x -v --timeout 280 --timeout-method thread > gpurun_out/mgpu_rehearsal_r06.log 2>&1 || { echo "rehearsal failed rc=$?"; tail -40 gpurun_out/mgpu_rehearsal_r06.log; exit 1; }
tail -2 gpurun_out/mgpu_rehearsal_r06.log
timeout -k 10 400 python -u tools/glass_lattice.py --out gpurun_out/glass_lattice_r06.json > gpurun_out/glass_lattice_r06.log 2>&1 || { echo "lattice failed rc=$?"; tail -20 gpurun_out/glass_lattice_r06.log; exit 1; }
cat gpurun_out/glass_lattice_r06.log
