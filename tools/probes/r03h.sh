#!/bin/bash
# round-3 probe 8: v7 epilogue cost split (stores vs GELU math); golden SDXL + pipelined DP tests
cd "${GRAFT_REPO_ROOT:-.}" || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest -q --timeout 120 --timeout-method thread tests/test_kernels_gpu.py \
   -k "gemm" > gpurun_out/r03h_kernels.log 2>&1 || { echo "kernel tests failed"; exit 1; }
AB_VARIANTS=0,8,128,136 timeout -k 10 300 python -u tools/probes/v7_ab.py > gpurun_out/r03h_ab.log 2>&1 || exit $?
timeout -k 10 300 python -u -m pytest -v --timeout 240 --timeout-method thread \
  tests/test_graphs_gpu.py -k "run_graph_with_model_patches" > gpurun_out/r03h_patches.log 2>&1
echo "patches rc=$?"
timeout -k 10 700 python -u -m pytest -v --timeout 300 --timeout-method thread \
  tests/test_golden_sdxl_gpu.py tests/test_dp_pipeline_gpu.py > gpurun_out/r03h_pytest.log 2>&1
echo "pytest rc=$?"
exit 0
