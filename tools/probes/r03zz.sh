#!/bin/bash
# round-3 probe 31: attention O epilogue with s_setprio around P.V: tests + A/B
cd "${GRAFT_REPO_ROOT:-.}" || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 400 python -u -m pytest -q -x --timeout 120 --timeout-method thread tests/ -m gpu -k "attn or attention" > gpurun_out/r03zz_tests.log 2>&1 || { echo "tests failed"; tail -30 gpurun_out/r03zz_tests.log; exit 1; }
tail -1 gpurun_out/r03zz_tests.log
timeout -k 10 300 python -u tools/probes/attn_prio_ab.py > gpurun_out/r03zz_ab.log 2>&1
rc=$?; echo "ab rc=$rc"; grep -v amdgpu.ids gpurun_out/r03zz_ab.log; exit $rc
