#!/bin/bash
# round-3 probe 32: re-tune every kernel choice with the current kernels (packaged table off), then the
# BASELINE configs 2-4 and the headline with the new table
cd "${GRAFT_REPO_ROOT:-.}" || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp HSA_ENABLE_IPC_MODE_LEGACY=0
export CGS_TUNE_FILE=gpurun_out/r03zj_tune.json
CGS_TUNE_DEFAULT=0 CGS_TUNE_REPS=5 timeout -k 10 500 python -u bench.py --steps 2 --warmup 2 > gpurun_out/r03zj_tune_bench.log 2>&1 || { echo "tune bench failed"; tail -20 gpurun_out/r03zj_tune_bench.log; exit 1; }
echo "tuned headline shapes: $(python -c 'import json;print(len(json.load(open("gpurun_out/r03zj_tune.json"))))')"
CGS_TUNE_DEFAULT=0 CGS_TUNE_REPS=5 timeout -k 10 900 python -u -m comfy_gen_server_amd.tools.bench_configs --which all --reps 1 > gpurun_out/r03zj_tune_configs.log 2>&1 || { echo "tune configs failed"; tail -20 gpurun_out/r03zj_tune_configs.log; exit 1; }
echo "tuned all shapes: $(python -c 'import json;print(len(json.load(open("gpurun_out/r03zj_tune.json"))))')"
