TAG=r01 bash tools/profile.sh && timeout -k 10 300 python bench.py > gpurun_out/bench_full.log 2>&1; tail -1 gpurun_out/bench_full.log
