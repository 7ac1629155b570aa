#!/bin/bash
# round-3 final check: v6 GEGLU A/B, full GPU tier, smoke, headline bench, rocprof table
cd "${GRAFT_REPO_ROOT:-.}" || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 900 python -u -m comfy_gen_server_amd.tools.bench_configs --which all --reps 2 > gpurun_out/${TAG:-r03zs}_configs.log 2>&1
echo "configs rc=$?"; grep "\"config\"" gpurun_out/${TAG:-r03zs}_configs.log | cut -c1-160
TAG=${TAG:-r03zs} bash tools/gpu_check.sh all || exit $?
PROF_STEPS=2 TAG=${TAG:-r03zs} bash tools/gpu_check.sh prof
