mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_kernels_gpu.py tests/test_graphs_gpu.py -x -q -k "dual or skip_concat or step_graph" --timeout 200 --timeout-method thread > gpurun_out/r02k_tests.log 2>&1 || exit $?
export CGS_TUNE_FILE=gpurun_out/tune_r02k.json TAG=r02k BENCH_ARGS="--steps 3 --warmup 1"
tools/gpu_check.sh bench
