#!/bin/bash
# round-3 probe 26: v6 split DMAs + v6 for the fused QKV: GEMM/conv GPU tests, headline bench, rocprof table
cd "${GRAFT_REPO_ROOT:-.}" || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp HSA_ENABLE_IPC_MODE_LEGACY=0
T=${TAG:-r03zc}
timeout -k 10 400 python -u -m pytest -q -x --timeout 120 --timeout-method thread tests/test_kernels_gpu.py \
   -k "gemm or conv or lnfold or v6" > gpurun_out/${T}_tests.log 2>&1 || { echo "tests failed"; tail -30 gpurun_out/${T}_tests.log; exit 1; }
tail -1 gpurun_out/${T}_tests.log
timeout -k 10 600 python -u bench.py --steps 4 --warmup 2 > gpurun_out/${T}_bench.log 2>&1
echo "bench rc=$?"
grep '"metric"' gpurun_out/${T}_bench.log | cut -c1-300
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d /tmp/prof_$T -o run -- python3 bench.py --steps 2 --warmup 1 > gpurun_out/${T}_prof_run.log 2>&1
echo "prof rc=$?"
db=$(find /tmp/prof_$T -name "*results.db" | head -n1)
[ -n "$db" ] && python -m comfy_gen_server_amd.tools.rocprof_summary "$db" "gpurun_out/${T}_prof.md" --top 40 && head -30 gpurun_out/${T}_prof.md
