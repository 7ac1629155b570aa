#!/bin/bash
# round-3 probe 41: batch-1 LayerNorm-folded GEMM shapes on every candidate (v6 joins the under-filled set)
cd "${GRAFT_REPO_ROOT:-.}" || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 300 python -u tools/probes/lnfold_b1.py > gpurun_out/r03zt_lnfold.log 2>&1
rc=$?; echo "rc=$rc"; grep -v amdgpu.ids gpurun_out/r03zt_lnfold.log; exit $rc
