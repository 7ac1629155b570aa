#!/bin/bash
# Kernel-level profile of the headline bench (tuned dispatch table first, then rocprofv3 kernel trace).
R="$GRAFT_REPO_ROOT"
cd "$R"; mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
export CGS_TUNE_FILE="$R/gpurun_out/tune.json"
timeout -k 10 400 python -u bench.py --steps 1 --warmup 1 > gpurun_out/bench_tune.log 2>&1 || exit $?
cd /tmp && export TMPDIR=/tmp
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d "$R/gpurun_out/prof" -o run -- python -u "$R/bench.py" --steps 1 --warmup 1 > "$R/gpurun_out/prof.log" 2>&1
rc=$?; echo "prof rc=$rc" >> "$R/gpurun_out/status.txt"; exit $rc
