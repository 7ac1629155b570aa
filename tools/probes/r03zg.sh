#!/bin/bash
# round-3 probe 30: v7 main loop without the fragment-read drain in phases 2 / 3 (dbg bit 512)
cd "${GRAFT_REPO_ROOT:-.}" || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp HSA_ENABLE_IPC_MODE_LEGACY=0
AB_VARIANTS=0,512 timeout -k 10 400 python -u tools/probes/v7_ab.py > gpurun_out/r03zg_v7ab.log 2>&1
rc=$?; echo "v7ab rc=$rc"; grep -v amdgpu.ids gpurun_out/r03zg_v7ab.log; exit $rc
