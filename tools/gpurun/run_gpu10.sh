#!/bin/bash
R="$GRAFT_REPO_ROOT"; cd "$R"; mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 300 python -u -m pytest tests/test_image_kernels_gpu.py tests/test_cascade.py tests/test_upscale.py -m gpu -v --timeout 200 --timeout-method thread > gpurun_out/pytest10.log 2>&1
echo "pytest rc=$?" >> gpurun_out/status.txt
