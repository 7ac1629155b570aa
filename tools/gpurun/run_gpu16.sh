#!/bin/bash
R="$GRAFT_REPO_ROOT"; cd "$R"; mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -m gpu -x -q -k "fp8 or gemm" --timeout 200 --timeout-method thread > gpurun_out/pytest16.log 2>&1
echo "pytest rc=$?" >> gpurun_out/status.txt
