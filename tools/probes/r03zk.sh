#!/bin/bash
# round-3 probe 33: v6 column-tile-4 stores paired with v_permlane16_swap (16 B) vs 8 B: GEMM/conv tests + A/B
cd "${GRAFT_REPO_ROOT:-.}" || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 400 python -u -m pytest -q -x --timeout 120 --timeout-method thread tests/test_kernels_gpu.py -k "gemm or conv or lnfold or v6" > gpurun_out/r03zk_tests.log 2>&1 || { echo "tests failed"; tail -30 gpurun_out/r03zk_tests.log; exit 1; }
tail -1 gpurun_out/r03zk_tests.log
V6_MODES=1,33 V6_CONV_MODES=19,51 timeout -k 10 300 python -u tools/probes/v6_ab.py > gpurun_out/r03zk_v6ab.log 2>&1
rc=$?; echo "v6ab rc=$rc"; grep -v amdgpu.ids gpurun_out/r03zk_v6ab.log; exit $rc
