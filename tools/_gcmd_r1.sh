export CGS_AUTOTUNE=0
tools/gpu_steps.sh "600|pytest_gc|python -m pytest tests/test_kernels_gpu.py -x -q -k 'gemm or conv'" \
  "600|kbench_gemm|python -m comfy_gen_server_amd.tools.kbench --gemm"
