#!/bin/bash
# round-3 probe 11: GELU A/B (+LN-folded forms), headline bench check, batch-1 kernel profile
cd "${GRAFT_REPO_ROOT:-.}" || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest -q --timeout 120 --timeout-method thread tests/test_kernels_gpu.py \
   -k "gemm or geglu or lnfold or gelu" > gpurun_out/r03k_kernels.log 2>&1 || { echo "kernel tests failed"; tail -30 gpurun_out/r03k_kernels.log; exit 1; }
AB_VARIANTS=0,256 timeout -k 10 400 python -u tools/probes/v7_ab.py > gpurun_out/r03k_ab.log 2>&1 || exit $?
timeout -k 10 600 python -u bench.py --steps 3 --warmup 2 > gpurun_out/r03k_bench.log 2>&1 || { echo "bench failed"; tail -5 gpurun_out/r03k_bench.log; exit 1; }
tail -1 gpurun_out/r03k_bench.log
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d gpurun_out/r03k_b1prof -o run -- python3 bench.py --batch-per-gpu 1 --steps 3 --warmup 2 > gpurun_out/r03k_b1.log 2>&1
echo "b1 prof rc=$?"
tail -1 gpurun_out/r03k_b1.log
exit 0
