#!/bin/bash
R="$GRAFT_REPO_ROOT"; cd "$R"; mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -m gpu -x -v -k "wide or vae_mid or attention" --timeout 200 --timeout-method thread > gpurun_out/pytest6.log 2>&1
rc=$?; echo "pytest rc=$rc" >> gpurun_out/status.txt; [ $rc -ne 0 ] && exit $rc
CGS_STAGE_TIMING=1 timeout -k 10 480 python -u bench.py --steps 2 --warmup 1 --profile-ops > gpurun_out/bench6.log 2>&1
echo "bench rc=$?" >> gpurun_out/status.txt
