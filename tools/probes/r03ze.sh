#!/bin/bash
# round-3 probe 28: one-pass GN finalize (tests), GN statistics in the conv epilogue A/B
cd "${GRAFT_REPO_ROOT:-.}" || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 400 python -u -m pytest -q -x --timeout 120 --timeout-method thread tests/ -m gpu \
   -k "groupnorm or group_norm or gn_ or resblock or vae" > gpurun_out/r03ze_tests.log 2>&1 || { echo "tests failed"; tail -30 gpurun_out/r03ze_tests.log; exit 1; }
tail -1 gpurun_out/r03ze_tests.log
timeout -k 10 300 python -u tools/probes/gns_ab.py > gpurun_out/r03ze_gns.log 2>&1
rc=$?; echo "gns rc=$rc"; grep -v amdgpu.ids gpurun_out/r03ze_gns.log; [ $rc = 0 ] || exit $rc
V6_MODES=1,17,19 timeout -k 10 300 python -u tools/probes/v6_ab.py > gpurun_out/r03ze_v6ab.log 2>&1
rc=$?; echo "v6ab rc=$rc"; grep -v amdgpu.ids gpurun_out/r03ze_v6ab.log; exit $rc
