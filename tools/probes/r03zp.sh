#!/bin/bash
# round-3 probe 37: Stable Cascade Stage C GEMM shapes on every HIP variant
cd "${GRAFT_REPO_ROOT:-.}" || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 400 python -u tools/probes/casc_gemm.py > gpurun_out/r03zp_casc_gemm.log 2>&1
rc=$?; echo "rc=$rc"; grep -v amdgpu.ids gpurun_out/r03zp_casc_gemm.log; exit $rc
