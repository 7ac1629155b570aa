#!/bin/bash
# round-3 probe 42: GroupNorm pixel blocks capped at 256 per image (batch 1-2): tests + batch-1 config A/B
cd "${GRAFT_REPO_ROOT:-.}" || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 400 python -u -m pytest -q -x --timeout 120 --timeout-method thread tests/ -m gpu -k "groupnorm or group_norm or gn_ or vae" > gpurun_out/r03zv_tests.log 2>&1 || { echo "tests failed"; tail -30 gpurun_out/r03zv_tests.log; exit 1; }
tail -1 gpurun_out/r03zv_tests.log
for r in 1 2; do
  for nb in 100000 256; do
    CGS_GN_MAXNB=$nb timeout -k 10 300 python -u -m comfy_gen_server_amd.tools.bench_configs --which sdxl_b1 --reps 2 > gpurun_out/r03zv_b1_${nb}_$r.log 2>&1 || exit 1
    echo "maxnb=$nb round $r: $(grep '"config"' gpurun_out/r03zv_b1_${nb}_$r.log | cut -c1-90)"
  done
done
