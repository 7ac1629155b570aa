#!/bin/bash
# upscaler / face-restoration GPU tests, then the whole GPU tier
R="$GRAFT_REPO_ROOT"; cd "$R"; mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 600 python -u -m pytest tests/test_upscale.py -m gpu -v --timeout 300 --timeout-method thread > gpurun_out/pytest9_up.log 2>&1
rc=$?; echo "upscale rc=$rc" >> gpurun_out/status.txt; [ $rc -ne 0 ] && exit $rc
timeout -k 10 900 python -u -m pytest tests/ -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/pytest9.log 2>&1
echo "pytest rc=$?" >> gpurun_out/status.txt
