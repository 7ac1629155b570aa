#!/bin/bash
# round-3 probe 3: v7 full-line epilogue (LDS staging) -- correctness, then timing with stagger modes
cd "${GRAFT_REPO_ROOT:-.}" || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_kernels_gpu.py -x -q --timeout 120 --timeout-method thread \
   -k "gemm or conv or layernorm_folded or lnfold or skip_concat" > gpurun_out/r03c_pytest.log 2>&1 || exit $?
for d in 0 8 256 512 1024 272 528 0; do
  CGS_V7_SPLIT_DBG=$d timeout -k 10 120 python -u tools/probes/v7_dbg.py >> gpurun_out/r03c_v7dbg.log 2>&1 || exit $?
done
exit 0
