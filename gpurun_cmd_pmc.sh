TAG=a1 BENCH_ARGS="--steps 10 --warmup 2 --no-cpu" bash tools/pmc.sh \
 "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_THREAD_CYCLES_VALU" \
 "SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_SCA SQ_LEVEL_WAVES SQ_INSTS_LDS SQ_INSTS_SMEM SQ_INSTS_BRANCH" \
 "TCC_HIT_sum TCC_MISS_sum GRBM_GUI_ACTIVE GRBM_COUNT TCP_TOTAL_CACHE_ACCESSES_sum TCP_TCC_READ_REQ_sum" && \
python tools/pmc_report.py gpurun_out/pmc_a1 "k_render<1, false, false, true>" > gpurun_out/pmc_a1_ext.txt && \
python tools/pmc_report.py gpurun_out/pmc_a1 "k_render<1, false, false, false>" > gpurun_out/pmc_a1_v1.txt && cat gpurun_out/pmc_a1_ext.txt gpurun_out/pmc_a1_v1.txt
