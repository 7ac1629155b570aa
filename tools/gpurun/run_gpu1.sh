#!/bin/bash
# GPU validation run: gpu tests, smoke, short bench. Stops at the first crash/timeout.
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
bad() { case "$1" in 124|134|137|139|143) return 0;; *) return 1;; esac; }
timeout -k 10 420 python -u -m pytest tests -m gpu -x -q --timeout 240 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc" >> gpurun_out/status.txt; bad $rc && exit $rc
timeout -k 10 240 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1
rc=$?; echo "smoke rc=$rc" >> gpurun_out/status.txt; [ $rc -ne 0 ] && exit $rc
CGS_STAGE_TIMING=1 timeout -k 10 480 python -u bench.py --steps 2 --warmup 1 --profile-ops > gpurun_out/bench.log 2>&1
rc=$?; echo "bench rc=$rc" >> gpurun_out/status.txt
exit $rc
