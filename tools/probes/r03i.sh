#!/bin/bash
# round-3 probe 9: GELU forms in the v7 GEGLU epilogue; staged full-line plain stores with/without desync
cd "${GRAFT_REPO_ROOT:-.}" || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest -q --timeout 120 --timeout-method thread tests/test_kernels_gpu.py \
   -k "gemm or geglu or lnfold" > gpurun_out/r03i_kernels.log 2>&1 || { echo "kernel tests failed"; tail -30 gpurun_out/r03i_kernels.log; exit 1; }
AB_VARIANTS=0,256,512,128,8,1024,5120,4096 timeout -k 10 400 python -u tools/probes/v7_ab.py > gpurun_out/r03i_ab.log 2>&1 || exit $?
timeout -k 10 300 python -u -m pytest -v --timeout 240 --timeout-method thread tests/test_dp_pipeline_gpu.py > gpurun_out/r03i_dp.log 2>&1
echo "dp rc=$?"
exit 0
