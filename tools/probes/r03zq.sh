#!/bin/bash
# round-3 probe 38: split-K small-tile GEMM: tests + Cascade / SDXL-b1 shape table
cd "${GRAFT_REPO_ROOT:-.}" || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 400 python -u -m pytest -q -x --timeout 120 --timeout-method thread tests/test_kernels_gpu.py -k "split_k or gemm" > gpurun_out/r03zq_tests.log 2>&1 || { echo "tests failed"; tail -30 gpurun_out/r03zq_tests.log; exit 1; }
tail -1 gpurun_out/r03zq_tests.log
timeout -k 10 400 python -u tools/probes/casc_gemm.py > gpurun_out/r03zq_gemm.log 2>&1
rc=$?; echo "rc=$rc"; grep -v amdgpu.ids gpurun_out/r03zq_gemm.log; exit $rc
