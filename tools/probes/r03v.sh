#!/bin/bash
# round-3 probe 20: sigmoid-quintic GELU everywhere (GRN, GEGLU epilogues), native channel affine;
# Cascade config + ATen attribution; headline bench
cd "${GRAFT_REPO_ROOT:-.}" || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 400 python -u -m pytest -q -x --timeout 120 --timeout-method thread tests/test_image_kernels_gpu.py tests/test_kernels_gpu.py \
   -k "grn or geglu or gelu or channel_affine or gemm or cascade" > gpurun_out/r03v_tests.log 2>&1 || { echo "tests failed"; tail -30 gpurun_out/r03v_tests.log; exit 1; }
tail -1 gpurun_out/r03v_tests.log
CGS_TORCH_PROFILE=1 timeout -k 10 900 python -u -m comfy_gen_server_amd.tools.bench_configs --which cascade --reps 2 > gpurun_out/r03v_casc.log 2>&1
echo "cascade rc=$?"
grep -E '"config"|^ATEN' gpurun_out/r03v_casc.log | cut -c1-420
timeout -k 10 600 python -u bench.py --steps 4 --warmup 2 > gpurun_out/r03v_bench.log 2>&1
echo "bench rc=$?"
grep '"metric"' gpurun_out/r03v_bench.log | cut -c1-300
exit 0
