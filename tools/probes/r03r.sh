#!/bin/bash
# round-3 probe 17: attention row sums on the MFMA (numerics + speed), then the full GPU tier from the
# LoRA test onward, smoke, headline bench, steady-state profile
cd "${GRAFT_REPO_ROOT:-.}" || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 300 python -u -m pytest -q -x --timeout 120 --timeout-method thread tests/test_kernels_gpu.py -k "attention or flash" \
   > gpurun_out/r03r_attn.log 2>&1 || { echo "attention tests failed"; tail -30 gpurun_out/r03r_attn.log; exit 1; }
tail -1 gpurun_out/r03r_attn.log
TAG=r03r PROF_TAIL=8 tools/gpu_check.sh all prof
