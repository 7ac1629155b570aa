#!/bin/bash
# round-3 probe 34: SDXL batch-1 rocprof kernel table with the current build
cd "${GRAFT_REPO_ROOT:-.}" || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d /tmp/prof_b1 -o run -- python3 -m comfy_gen_server_amd.tools.bench_configs --which sdxl_b1 --reps 2 > gpurun_out/r03zu_casc.log 2>&1
echo "prof rc=$?"
grep '"config"' gpurun_out/r03zu_casc.log | cut -c1-200
db=$(find /tmp/prof_b1 -name "*results.db" | head -n1)
[ -n "$db" ] && python -m comfy_gen_server_amd.tools.rocprof_summary "$db" "gpurun_out/r03zu_b1_profile.md" --top 45 && head -50 gpurun_out/r03zu_b1_profile.md
