#!/bin/bash
# the other BASELINE configs on one MI355X (SDXL b1 latency, SDXL+ControlNet+LoRA, Cascade C->B->A)
R="$GRAFT_REPO_ROOT"; cd "$R"; mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
export CGS_TUNE_FILE="$R/gpurun_out/tune_cfg.json"
timeout -k 10 1000 python -u -m comfy_gen_server_amd.tools.bench_configs --which "${1:-all}" --reps 2 >> gpurun_out/bench_configs.log 2>&1
echo "configs rc=$?" >> gpurun_out/status.txt
