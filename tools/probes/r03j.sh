#!/bin/bash
# round-3 probe 10: sigmoid-quintic vs A&S GELU in the GEGLU epilogue (incl. LN-folded forms); bench check
cd "${GRAFT_REPO_ROOT:-.}" || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest -q --timeout 120 --timeout-method thread tests/test_kernels_gpu.py \
   -k "gemm or geglu or lnfold or gelu" > gpurun_out/r03j_kernels.log 2>&1 || { echo "kernel tests failed"; tail -30 gpurun_out/r03j_kernels.log; exit 1; }
AB_VARIANTS=0,256 timeout -k 10 400 python -u tools/probes/v7_ab.py > gpurun_out/r03j_ab.log 2>&1 || exit $?
timeout -k 10 600 python -u bench.py --steps 3 --warmup 2 > gpurun_out/r03j_bench.log 2>&1
echo "bench rc=$?"
tail -2 gpurun_out/r03j_bench.log
exit 0
