#!/bin/bash
R="$GRAFT_REPO_ROOT"; cd "$R"; mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py tests/test_runtime_native.py -m gpu -x -q -k "groupnorm or hbm or unet or resblock" --timeout 200 --timeout-method thread > gpurun_out/pytest13.log 2>&1
rc=$?; echo "pytest rc=$rc" >> gpurun_out/status.txt; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke13.log 2>&1
echo "smoke rc=$?" >> gpurun_out/status.txt
