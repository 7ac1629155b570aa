#!/bin/bash
R="$GRAFT_REPO_ROOT"; cd "$R"; mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -m gpu -x -q -k "attention_d64" --timeout 200 --timeout-method thread > gpurun_out/pytest15.log 2>&1
rc=$?; echo "pytest rc=$rc" >> gpurun_out/status.txt; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python -u -m comfy_gen_server_amd.tools.kbench --attn > gpurun_out/kbench_attn15.log 2>&1
echo "kbench rc=$?" >> gpurun_out/status.txt
