#!/bin/bash
# round-3 probe 36: two-source K/V attention + fused QKV/KV projections for Stable Cascade self-attention
cd "${GRAFT_REPO_ROOT:-.}" || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 500 python -u -m pytest -q -x --timeout 120 --timeout-method thread tests/ -m gpu -k "attention or attn or cascade or grn" > gpurun_out/r03zo_tests.log 2>&1 || { echo "tests failed"; tail -30 gpurun_out/r03zo_tests.log; exit 1; }
tail -1 gpurun_out/r03zo_tests.log
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d /tmp/prof_casc2 -o run -- python3 -m comfy_gen_server_amd.tools.bench_configs --which cascade --reps 2 > gpurun_out/r03zo_casc.log 2>&1
echo "prof rc=$?"
grep '"config"' gpurun_out/r03zo_casc.log | cut -c1-200
db=$(find /tmp/prof_casc2 -name "*results.db" | head -n1)
[ -n "$db" ] && python -m comfy_gen_server_amd.tools.rocprof_summary "$db" "gpurun_out/r03zo_cascade_profile.md" --top 45 && head -30 gpurun_out/r03zo_cascade_profile.md
