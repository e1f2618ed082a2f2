cd "${GRAFT_REPO_ROOT}" && mkdir -p gpurun_out && \
timeout -k 10 300 python tools/abtime.py --config C3 --flags 0,48 --rounds 9 old=build/variants/old.so new=voxmap_amd/libvoxmap_hip.so > gpurun_out/ab_c3.log 2>&1 && cat gpurun_out/ab_c3.log && \
timeout -k 10 400 python tools/abtime.py --config C5 --flags 48 --rounds 5 --frames 10 old=build/variants/old.so new=voxmap_amd/libvoxmap_hip.so > gpurun_out/ab_c5.log 2>&1 && cat gpurun_out/ab_c5.log
