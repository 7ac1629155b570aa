#!/bin/bash
# round-3 probe 19: attention two-deep staging (tests + TF/s), then BASELINE configs 2-4 and a Cascade
# kernel profile with the current build
cd "${GRAFT_REPO_ROOT:-.}" || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 300 python -u -m pytest -q -x --timeout 120 --timeout-method thread tests/test_kernels_gpu.py -k "attention or flash" \
   > gpurun_out/r03u_attn.log 2>&1 || { echo "attention tests failed"; tail -30 gpurun_out/r03u_attn.log; exit 1; }
tail -1 gpurun_out/r03u_attn.log
timeout -k 10 200 python -u tools/probes/attn_bench.py 2>&1 | grep -v amdgpu.ids | tee gpurun_out/r03u_attn_bench.log
timeout -k 10 900 python -u -m comfy_gen_server_amd.tools.bench_configs --which all --reps 2 > gpurun_out/r03u_configs.log 2>&1
echo "configs rc=$?"
grep '"config"' gpurun_out/r03u_configs.log | cut -c1-260
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d /tmp/r03u_casc -o run -- python3 -m comfy_gen_server_amd.tools.bench_configs --which cascade --reps 1 > gpurun_out/r03u_casc.log 2>&1
echo "cascade prof rc=$?"
db=$(find /tmp/r03u_casc -name "*results.db" | head -n1)
[ -n "$db" ] && python -m comfy_gen_server_amd.tools.rocprof_summary "$db" gpurun_out/r03u_cascade_prof.md --top 45 > /dev/null && head -30 gpurun_out/r03u_cascade_prof.md
exit 0
