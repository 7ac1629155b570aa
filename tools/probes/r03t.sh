#!/bin/bash
# round-3 probe 18: attention with two-deep K/V register staging (numerics + TF/s)
cd "${GRAFT_REPO_ROOT:-.}" || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest -q -x --timeout 120 --timeout-method thread tests/test_kernels_gpu.py -k "attention or flash" \
   > gpurun_out/r03t_attn.log 2>&1 || { echo "attention tests failed"; tail -30 gpurun_out/r03t_attn.log; exit 1; }
tail -1 gpurun_out/r03t_attn.log
timeout -k 10 200 python -u tools/probes/attn_bench.py 2>&1 | grep -v amdgpu.ids
