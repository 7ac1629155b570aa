#!/bin/bash
R="$GRAFT_REPO_ROOT"; cd "$R"; mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 300 python -u -m comfy_gen_server_amd.tools.kbench --gemm > gpurun_out/kbench_gemm.log 2>&1
echo "kbench rc=$?" >> gpurun_out/status.txt
