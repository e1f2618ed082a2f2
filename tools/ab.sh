#!/bin/bash
# A/B timing of kernel variants: each argument is "label:VAR=val,VAR=val".
# e.g. tools/ab.sh single:VOXMAP_PAIR=0 b221:VOXMAP_PAIR=0,VOXMAP_LIB=build/variants/b221.so
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for spec in "$@"; do
  label=${spec%%:*}; envs=${spec#*:}
  for f in ${AB_FLAGS:-0 8}; do
    env ${envs//,/ } timeout -k 10 120 python bench.py --no-cpu --steps 30 --warmup 3 --flags $f ${AB_ARGS} > gpurun_out/ab.log 2>&1 || { tail -20 gpurun_out/ab.log; exit 1; }
    echo "$label flags=$f $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/ab.log)"
  done
done
