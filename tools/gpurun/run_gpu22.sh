#!/bin/bash
# GroupNorm finalize/apply rewrite: kernel tests, then a profiled bench (tuned table first)
R="$GRAFT_REPO_ROOT"; cd "$R"; mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -m gpu -x -q -k "groupnorm or layernorm" --timeout 200 --timeout-method thread > gpurun_out/pytest22.log 2>&1
rc=$?; echo "pytest rc=$rc" >> gpurun_out/status.txt; [ $rc -ne 0 ] && exit $rc
bash tools/gpurun/run_gpu_prof.sh
