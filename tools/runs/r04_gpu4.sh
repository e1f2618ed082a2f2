#!/bin/bash
# round 4: bisect the v1 / full-quality regression against the round-3 head with
# lean A/B builds (VX_AB_LEAN: untiled RGBA8 kernels only): the head, the r03
# shading block (VX_OLD_SHADE), no quad split (VX_NO_QUAD, VX_QSPEC=0), both;
# then the pooled soft-shadow pass on C5 (flags 0x80) with its block times.
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/../.." && pwd)}"
cd "$ROOT"; mkdir -p gpurun_out
timeout -k 10 500 python tools/abtime.py --config C3 --flags 48,0 --rounds 7 head=ab/lean_head.so oldshade=ab/lean_oldshade.so noquad=ab/lean_noquad.so both=ab/lean_both.so r03=ab/lib_r03.so > gpurun_out/ab_bisect_c3.txt 2>&1 || { echo "ab c3 failed"; tail gpurun_out/ab_bisect_c3.txt; exit 1; }
cat gpurun_out/ab_bisect_c3.txt
timeout -k 10 400 python tools/abtime.py --config C5 --flags 48,176 --rounds 3 --frames 10 new=voxmap_amd/libvoxmap_hip.so > gpurun_out/ab_pool_c5.txt 2>&1 || { echo "ab c5 failed"; tail gpurun_out/ab_pool_c5.txt; exit 1; }
cat gpurun_out/ab_pool_c5.txt
timeout -k 10 200 python tools/block_times.py ab/lib_btime.so --config C5 --flags 176 --out gpurun_out/btime_c5_pool.json > gpurun_out/btime_c5_pool.log 2>&1 || { echo "btime failed"; tail gpurun_out/btime_c5_pool.log; exit 1; }
python -c "
import json
d=json.load(open('gpurun_out/btime_c5_pool.json'))
for f in d['frames'][:2]: print('c5 pool', {k:v for k,v in f.items() if k!='row_mean_us'})
"
