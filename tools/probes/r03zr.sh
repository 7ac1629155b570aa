#!/bin/bash
# round-3 probe 39: GEGLU on v6 (tests + A/B vs v7), Cascade two-source model test
cd "${GRAFT_REPO_ROOT:-.}" || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 500 python -u -m pytest -q -x --timeout 120 --timeout-method thread tests/test_kernels_gpu.py -k "geglu or lnfold or layernorm_folded or cascade or two_source or two_kv" > gpurun_out/r03zr_tests.log 2>&1 || { echo "tests failed"; tail -40 gpurun_out/r03zr_tests.log; exit 1; }
tail -1 gpurun_out/r03zr_tests.log
timeout -k 10 300 python -u tools/probes/geglu_v6.py > gpurun_out/r03zr_ab.log 2>&1
rc=$?; echo "ab rc=$rc"; grep -v amdgpu.ids gpurun_out/r03zr_ab.log; exit $rc
