#!/bin/bash
# round-3 probe 1: store shapes, current GEMM table, hipBLASLt kernel names
cd "${GRAFT_REPO_ROOT:-.}" || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 120 tools/probes/store_probe > gpurun_out/r03a_store.log 2>&1 || exit $?
timeout -k 10 400 python -u -m comfy_gen_server_amd.tools.gemm_table gpurun_out/r03a_gemm.md > gpurun_out/r03a_gemm.log 2>&1 || exit $?
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d /tmp/r03a_lib -o run -- python3 tools/probes/lib_gemm_names.py > gpurun_out/r03a_lib.log 2>&1 || exit $?
f=$(find /tmp/r03a_lib -name "*kernel_stats.csv" | head -n1)
[ -n "$f" ] && cp "$f" gpurun_out/r03a_lib_kernel_stats.csv
exit 0
