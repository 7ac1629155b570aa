#!/bin/bash
# round-3 probe 13: small-tile GEMM variants (v10 64x128, v11 128x64, LN fold on v8/v10/v11) for batch-1 grids
cd "${GRAFT_REPO_ROOT:-.}" || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest -q -x --timeout 120 --timeout-method thread tests/test_kernels_gpu.py \
   -k "gemm or lnfold or layernorm_folded or attention or groupnorm" > gpurun_out/r03m_kernels.log 2>&1 || { echo "kernel tests failed"; tail -30 gpurun_out/r03m_kernels.log; exit 1; }
tail -1 gpurun_out/r03m_kernels.log
timeout -k 10 300 python -u tools/probes/small_m.py > gpurun_out/r03m_smallm.log 2>&1 || { echo "small_m failed"; tail -20 gpurun_out/r03m_smallm.log; exit 1; }
cat gpurun_out/r03m_smallm.log | grep -v amdgpu.ids
timeout -k 10 600 python -u bench.py --batch-per-gpu 1 --steps 3 --warmup 2 > gpurun_out/r03m_b1.log 2>&1 || { echo "b1 bench failed"; tail -5 gpurun_out/r03m_b1.log; exit 1; }
grep '"metric"' gpurun_out/r03m_b1.log | cut -c1-330
exit 0
