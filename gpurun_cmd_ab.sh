mkdir -p gpurun_out
timeout -k 10 200 python tools/enqueue_rate.py --flags 48 || exit 1
timeout -k 10 200 python tools/enqueue_rate.py --flags 0 || exit 1
timeout -k 10 300 python bench.py --no-cpu > gpurun_out/b.log 2>&1 || { tail -5 gpurun_out/b.log; exit 1; }
tail -1 gpurun_out/b.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['ms_per_step'], d['roofline']['avg_launch_ms'], d['roofline']['frac'], d['config']['v1'])"
