#!/bin/bash
# Frame time with parts of the shading switched off (VX_FLAG_* bits), one process each.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for f in 0 1 2 4 7 8; do
  timeout -k 10 120 python bench.py --no-cpu --steps 30 --warmup 3 --flags $f > gpurun_out/ablate_$f.log 2>&1 || exit $?
  echo "flags=$f $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/ablate_$f.log)"
done
