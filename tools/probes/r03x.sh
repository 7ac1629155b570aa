#!/bin/bash
# round-3 probe 22: GRN finalize over a (C/256, N) grid, mean formed in the apply pass
cd "${GRAFT_REPO_ROOT:-.}" || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 300 python -u -m pytest -q -x --timeout 120 --timeout-method thread tests/test_image_kernels_gpu.py tests/test_graphs_gpu.py \
   -k "grn or cascade" > gpurun_out/r03x_tests.log 2>&1 || { echo "tests failed"; tail -30 gpurun_out/r03x_tests.log; exit 1; }
tail -1 gpurun_out/r03x_tests.log
timeout -k 10 900 python -u -m comfy_gen_server_amd.tools.bench_configs --which cascade --reps 2 > gpurun_out/r03x_casc.log 2>&1
echo "cascade rc=$?"
grep '"config"' gpurun_out/r03x_casc.log | cut -c1-200
