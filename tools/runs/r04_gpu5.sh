#!/bin/bash
# round 4: the simple shading block restored for EXT 1/2 (the general loop only in
# EXT 5/6) against the round-3 head; block rows bottom-up (0x4000) single stream;
# per-block times of C5 in both orders; every GPU test.
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/../.." && pwd)}"
cd "$ROOT"; mkdir -p gpurun_out
timeout -k 10 500 python tools/abtime.py --config C3 --flags 48,16432,0,16384 --rounds 7 new=voxmap_amd/libvoxmap_hip.so r03=ab/lib_r03.so > gpurun_out/ab_fix_c3.txt 2>&1 || { echo "ab c3 failed"; tail gpurun_out/ab_fix_c3.txt; exit 1; }
cat gpurun_out/ab_fix_c3.txt
timeout -k 10 500 python tools/abtime.py --config C5 --flags 48,16432 --rounds 3 --frames 10 new=voxmap_amd/libvoxmap_hip.so r03=ab/lib_r03.so > gpurun_out/ab_fix_c5.txt 2>&1 || { echo "ab c5 failed"; tail gpurun_out/ab_fix_c5.txt; exit 1; }
cat gpurun_out/ab_fix_c5.txt
for fl in 48 16432; do
timeout -k 10 200 python tools/block_times.py ab/lib_btime.so --config C5 --flags $fl --out gpurun_out/btime_c5_$fl.json > gpurun_out/btime_c5_$fl.log 2>&1 || { echo "btime failed"; tail gpurun_out/btime_c5_$fl.log; exit 1; }
done
python -c "
import json
for fl in (48, 16432):
    d=json.load(open('gpurun_out/btime_c5_%d.json'%fl))
    for f in d['frames'][:2]: print('c5', fl, {k:v for k,v in f.items() if k!='row_mean_us'})
"
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1
rc=$?; tail -3 gpurun_out/pytest_gpu.log; exit $rc
