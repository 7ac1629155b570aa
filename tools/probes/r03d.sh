#!/bin/bash
# round-3 probe 4: in-process A/B of the v7 epilogue variants
cd "${GRAFT_REPO_ROOT:-.}" || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp
AB_VARIANTS=0,32,8,40 timeout -k 10 300 python -u tools/probes/v7_ab.py > gpurun_out/r03d_ab.log 2>&1 || exit $?
exit 0
