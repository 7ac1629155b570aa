#!/bin/bash
R="$GRAFT_REPO_ROOT"; cd "$R"; mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 400 python -u -m comfy_gen_server_amd.tools.kbench > gpurun_out/kbench_full.log 2>&1
echo "kbench rc=$?" >> gpurun_out/status.txt
