#!/bin/bash
# round 6, end: sanity A/B of the product against the measured variant
# (ab/doom_hard.so), then the profiles, the bench line and the GPU suite
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/../.." && pwd)}"
cd "$ROOT"; mkdir -p gpurun_out
L=voxmap_amd/libvoxmap_hip.so
timeout -k 10 300 python -u tools/abtime.py --config C3 --flags 48 --rounds 5 --frames 20 head=$L variant=ab/doom_hard.so > gpurun_out/ab_final_sanity.txt 2>&1 || { echo "sanity ab failed"; tail -20 gpurun_out/ab_final_sanity.txt; exit 1; }
cat gpurun_out/ab_final_sanity.txt
bash tools/runs/r06_final.sh || exit 1
TAG=r06_end3 bash tools/runs/r06_gpu_tests.sh
