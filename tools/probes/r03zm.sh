#!/bin/bash
# round-3 probe 35: GRN apply with a parallel per-image prologue: GRN / Cascade tests + Cascade configs
cd "${GRAFT_REPO_ROOT:-.}" || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 400 python -u -m pytest -q -x --timeout 120 --timeout-method thread tests/ -m gpu -k "grn or cascade" > gpurun_out/r03zm_tests.log 2>&1 || { echo "tests failed"; tail -30 gpurun_out/r03zm_tests.log; exit 1; }
tail -1 gpurun_out/r03zm_tests.log
timeout -k 10 600 python -u -m comfy_gen_server_amd.tools.bench_configs --which cascade --reps 2 > gpurun_out/r03zm_casc.log 2>&1
echo "cascade rc=$?"
grep '"config"' gpurun_out/r03zm_casc.log | cut -c1-200
