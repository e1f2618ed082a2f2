#!/bin/bash
# round 6: the base colour and AO sample after the sun march (ab/ao_late.so) against the head
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/../.." && pwd)}"
cd "$ROOT"; mkdir -p gpurun_out
L=voxmap_amd/libvoxmap_hip.so
timeout -k 10 400 python -u tools/abtime.py --config C3 --flags 48,0 --rounds 11 --frames 20 head=$L late=ab/ao_late.so > gpurun_out/ab_aolate_c3.txt 2>&1 || { echo "c3 ab failed"; tail -20 gpurun_out/ab_aolate_c3.txt; exit 1; }
cat gpurun_out/ab_aolate_c3.txt
timeout -k 10 400 python -u tools/abtime.py --config C5 --flags 48 --rounds 5 --frames 10 head=$L late=ab/ao_late.so > gpurun_out/ab_aolate_c5.txt 2>&1 || { echo "c5 ab failed"; tail -20 gpurun_out/ab_aolate_c5.txt; exit 1; }
cat gpurun_out/ab_aolate_c5.txt
