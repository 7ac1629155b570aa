#!/bin/bash
R="$GRAFT_REPO_ROOT"; cd "$R"; mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 400 python -u -m pytest tests/test_e2e_gpu.py tests/test_runtime_native.py -m gpu -v --timeout 300 --timeout-method thread > gpurun_out/pytest11.log 2>&1
echo "pytest rc=$?" >> gpurun_out/status.txt
