#!/bin/bash
# round-3 probe 6: v7 A1 pre-issue (dbg 0) vs round-2 issue point (dbg 64); GEMM/conv correctness; new GPU tests
cd "${GRAFT_REPO_ROOT:-.}" || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest -q --timeout 120 --timeout-method thread tests/test_kernels_gpu.py \
   -k "gemm or conv or layernorm_folded or lnfold or skip_concat" > gpurun_out/r03f_kernels.log 2>&1 || { echo "kernel tests failed"; exit 1; }
AB_VARIANTS=0,64,8 timeout -k 10 300 python -u tools/probes/v7_ab.py > gpurun_out/r03f_ab.log 2>&1 || exit $?
timeout -k 10 700 python -u -m pytest -v --timeout 240 --timeout-method thread \
  tests/test_graphs_gpu.py tests/test_golden_sdxl_gpu.py tests/test_dp_pipeline_gpu.py > gpurun_out/r03f_pytest.log 2>&1
echo "pytest rc=$?"
exit 0
