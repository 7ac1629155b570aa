#!/bin/bash
# round-3 probe 24: v6 DMA placement A/B, column-split hybrid for 1.25-round GEMMs
cd "${GRAFT_REPO_ROOT:-.}" || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 500 python -u tools/probes/qkv_ab.py > gpurun_out/r03zb_qkv.log 2>&1
rc=$?; echo "qkv_ab rc=$rc"; cat gpurun_out/r03zb_qkv.log | grep -v amdgpu.ids
exit $rc
