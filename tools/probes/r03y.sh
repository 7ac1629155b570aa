#!/bin/bash
# round-3 probe 23: depthwise conv / nearest upsample with 32-bit index math; configs 2-4; headline
cd "${GRAFT_REPO_ROOT:-.}" || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 400 python -u -m pytest -q -x --timeout 120 --timeout-method thread tests/test_kernels_gpu.py tests/test_image_kernels_gpu.py \
   -k "dw or depthwise or upsample or elementwise or grn or cascade" > gpurun_out/r03y_tests.log 2>&1 || { echo "tests failed"; tail -30 gpurun_out/r03y_tests.log; exit 1; }
tail -1 gpurun_out/r03y_tests.log
timeout -k 10 900 python -u -m comfy_gen_server_amd.tools.bench_configs --which all --reps 2 > gpurun_out/r03y_configs.log 2>&1
echo "configs rc=$?"
grep '"config"' gpurun_out/r03y_configs.log | cut -c1-200
timeout -k 10 600 python -u bench.py --steps 4 --warmup 2 > gpurun_out/r03y_bench.log 2>&1
echo "bench rc=$?"
grep '"metric"' gpurun_out/r03y_bench.log | cut -c1-260
