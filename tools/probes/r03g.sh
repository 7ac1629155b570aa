#!/bin/bash
# round-3 probe 7: v7 start-phase desync (8 phases per XCD) vs synchronized rounds; remaining GPU tests
cd "${GRAFT_REPO_ROOT:-.}" || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest -q --timeout 120 --timeout-method thread tests/test_kernels_gpu.py \
   -k "gemm" > gpurun_out/r03g_kernels.log 2>&1 || { echo "kernel tests failed"; exit 1; }
AB_VARIANTS=0,8,288,304,544,296,64 timeout -k 10 400 python -u tools/probes/v7_ab.py > gpurun_out/r03g_ab.log 2>&1 || exit $?
timeout -k 10 700 python -u -m pytest -v --timeout 240 --timeout-method thread \
  tests/test_graphs_gpu.py -k "run_graph" tests/test_golden_sdxl_gpu.py tests/test_dp_pipeline_gpu.py > gpurun_out/r03g_pytest.log 2>&1
echo "pytest rc=$?"
exit 0
