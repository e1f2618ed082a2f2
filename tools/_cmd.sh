cd "${GRAFT_REPO_ROOT}" && mkdir -p gpurun_out && \
PYTEST_ARGS="--timeout 120 --timeout-method thread" BENCH_ARGS="--no-cpu" bash tools/gpu_check.sh
