#!/bin/bash
# full GPU test tier + smoke (what the driver runs at round end)
R="$GRAFT_REPO_ROOT"; cd "$R"; mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 900 python -u -m pytest tests/ -m gpu -x -v --timeout 200 --timeout-method thread > gpurun_out/pytest8.log 2>&1
rc=$?; echo "pytest rc=$rc" >> gpurun_out/status.txt; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke8.log 2>&1
echo "smoke rc=$?" >> gpurun_out/status.txt
