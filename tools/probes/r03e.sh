#!/bin/bash
# round-3 probe 5: v7 epilogue A/B, then the new GPU tests (run-graph samplers/patches, UNet dtypes)
cd "${GRAFT_REPO_ROOT:-.}" || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp
AB_VARIANTS=0,32,8,40 timeout -k 10 300 python -u tools/probes/v7_ab.py > gpurun_out/r03e_ab.log 2>&1 || exit $?
timeout -k 10 600 python -u -m pytest -v --timeout 240 --timeout-method thread \
  tests/test_unet_dtypes_gpu.py tests/test_graphs_gpu.py tests/test_rng_gpu.py tests/test_golden_sdxl_gpu.py tests/test_dp_pipeline_gpu.py > gpurun_out/r03e_pytest.log 2>&1
echo "pytest rc=$?"
exit 0
