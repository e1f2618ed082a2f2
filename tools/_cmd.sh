bash tools/gpu_check.sh && bash tools/ablate.sh && \
TAG=full bash tools/pmc.sh "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_VMEM_RD" "SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU" "TCC_HIT_sum TCC_MISS_sum GRBM_GUI_ACTIVE"
