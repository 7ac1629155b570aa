tools/gpu_steps.sh "600|pytest_gc|env CGS_AUTOTUNE=0 python -m pytest tests/test_kernels_gpu.py -x -q -k 'gemm or conv'" \
  "600|kbench_gemm|env CGS_AUTOTUNE=0 python -m comfy_gen_server_amd.tools.kbench --gemm" \
  "900|bench20|env CGS_TUNE_FILE=gpurun_out/tune.json python bench.py --steps 2 --warmup 1"
