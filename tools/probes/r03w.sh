#!/bin/bash
# round-3 probe 21: Cascade LayerNorm folded into the channel-MLP GEMM (numerics + config timing + profile)
cd "${GRAFT_REPO_ROOT:-.}" || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 300 python -u -m pytest -q -x --timeout 120 --timeout-method thread tests/test_kernels_gpu.py tests/test_graphs_gpu.py \
   -k "cascade or lnfold or layernorm_folded" > gpurun_out/r03w_tests.log 2>&1 || { echo "tests failed"; tail -30 gpurun_out/r03w_tests.log; exit 1; }
tail -1 gpurun_out/r03w_tests.log
timeout -k 10 900 python -u -m comfy_gen_server_amd.tools.bench_configs --which cascade --reps 2 > gpurun_out/r03w_casc.log 2>&1
echo "cascade rc=$?"
grep '"config"' gpurun_out/r03w_casc.log | cut -c1-200
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d /tmp/r03w_casc -o run -- python3 -m comfy_gen_server_amd.tools.bench_configs --which cascade --reps 1 > gpurun_out/r03w_cascprof.log 2>&1
echo "cascade prof rc=$?"
db=$(find /tmp/r03w_casc -name "*results.db" | head -n1)
[ -n "$db" ] && python -m comfy_gen_server_amd.tools.rocprof_summary "$db" gpurun_out/r03w_cascade_prof.md --top 45 > /dev/null && head -32 gpurun_out/r03w_cascade_prof.md
exit 0
