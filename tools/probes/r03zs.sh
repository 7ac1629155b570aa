#!/bin/bash
# round-3 final check: v6 GEGLU A/B, full GPU tier, smoke, headline bench, rocprof table
cd "${GRAFT_REPO_ROOT:-.}" || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 300 python -u tools/probes/geglu_v6.py > gpurun_out/r03zs_geglu_ab.log 2>&1
echo "geglu ab rc=$?"; grep -v amdgpu.ids gpurun_out/r03zs_geglu_ab.log
TAG=r03zs bash tools/gpu_check.sh all || exit $?
PROF_STEPS=2 TAG=r03zs bash tools/gpu_check.sh prof
