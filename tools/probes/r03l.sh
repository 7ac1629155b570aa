#!/bin/bash
# round-3 probe 12: headline bench with the arena fix, batch-1 kernel profile, arena GPU tests
cd "${GRAFT_REPO_ROOT:-.}" || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 200 python -u -m pytest -q --timeout 120 --timeout-method thread tests/test_weight_arena.py > gpurun_out/r03l_arena.log 2>&1 || { echo "arena tests failed"; tail -20 gpurun_out/r03l_arena.log; exit 1; }
timeout -k 10 600 python -u bench.py --steps 3 --warmup 2 > gpurun_out/r03l_bench.log 2>&1 || { echo "bench failed"; tail -5 gpurun_out/r03l_bench.log; exit 1; }
tail -1 gpurun_out/r03l_bench.log
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d gpurun_out/r03l_b1prof -o run -- python3 bench.py --batch-per-gpu 1 --steps 3 --warmup 2 > gpurun_out/r03l_b1.log 2>&1
echo "b1 prof rc=$?"
tail -1 gpurun_out/r03l_b1.log
exit 0
