#!/bin/bash
# round-end style check: full GPU tier, smoke, headline bench (default contract args)
R="$GRAFT_REPO_ROOT"; cd "$R"; mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 900 python -u -m pytest tests/ -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/pytest23.log 2>&1
rc=$?; echo "pytest rc=$rc" >> gpurun_out/status.txt; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke23.log 2>&1
rc=$?; echo "smoke rc=$rc" >> gpurun_out/status.txt; [ $rc -ne 0 ] && exit $rc
timeout -k 10 600 python -u bench.py > gpurun_out/bench23.log 2>&1
echo "bench rc=$?" >> gpurun_out/status.txt
