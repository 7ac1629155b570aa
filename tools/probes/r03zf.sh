#!/bin/bash
# round-3 probe 29: v6 phase 0 without the fragment-read drain before its barrier
cd "${GRAFT_REPO_ROOT:-.}" || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp HSA_ENABLE_IPC_MODE_LEGACY=0
V6_MODES=1,17,19 timeout -k 10 300 python -u tools/probes/v6_ab.py > gpurun_out/r03zf_v6ab.log 2>&1
rc=$?; echo "v6ab rc=$rc"; grep -v amdgpu.ids gpurun_out/r03zf_v6ab.log; exit $rc
