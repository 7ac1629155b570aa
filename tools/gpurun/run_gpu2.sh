#!/bin/bash
R="$GRAFT_REPO_ROOT"; cd "$R"; mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
bad() { case "$1" in 124|134|137|139|143) return 0;; *) return 1;; esac; }
timeout -k 10 300 python -u -m pytest tests/test_graphs_gpu.py tests/test_kernels_gpu.py -m gpu -x -q -k "graph or attention or conv2d or elementwise" --timeout 200 --timeout-method thread > gpurun_out/pytest2.log 2>&1
rc=$?; echo "pytest rc=$rc" >> gpurun_out/status.txt; bad $rc && exit $rc
true
rc=$?; echo "kbench rc=$rc" >> gpurun_out/status.txt; bad $rc && exit $rc
CGS_STAGE_TIMING=1 timeout -k 10 480 python -u bench.py --steps 2 --warmup 1 --profile-ops > gpurun_out/bench2.log 2>&1
rc=$?; echo "bench rc=$rc" >> gpurun_out/status.txt
CGS_GRAPHS=0 CGS_STAGE_TIMING=1 timeout -k 10 480 python -u bench.py --steps 2 --warmup 1 --batch-per-gpu 1 > gpurun_out/bench2_b1_nograph.log 2>&1
CGS_STAGE_TIMING=1 timeout -k 10 480 python -u bench.py --steps 2 --warmup 1 --batch-per-gpu 1 > gpurun_out/bench2_b1_graph.log 2>&1
exit $rc
