#!/bin/bash
# round-3 probe 2: per-CU store rate, v7 without stores / with staggered starts, hipBLASLt kernel names
cd "${GRAFT_REPO_ROOT:-.}" || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 120 tools/probes/store_probe > gpurun_out/r03b_store.log 2>&1 || exit $?
for d in 0 8 256 768 1536 0; do
  CGS_V7_SPLIT_DBG=$d timeout -k 10 120 python -u tools/probes/v7_dbg.py >> gpurun_out/r03b_v7dbg.log 2>&1 || exit $?
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/r03b_lib -o run -- python3 tools/probes/lib_gemm_names.py > gpurun_out/r03b_lib.log 2>&1 || exit $?
f=$(find /tmp/r03b_lib -name "*kernel_stats.csv" | head -n1)
[ -n "$f" ] && cp "$f" gpurun_out/r03b_lib_kernel_stats.csv
exit 0
