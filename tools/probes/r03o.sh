#!/bin/bash
# round-3 probe 15: v7 split-K forced on the batch-1 / Cascade small-M shapes (S = 2, 4, 6)
cd "${GRAFT_REPO_ROOT:-.}" || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp
for S in 2 4 6; do
  echo "== CGS_V7_SPLIT_FORCE=$S" >> gpurun_out/r03o_split.log
  CGS_V7_SPLIT_FORCE=$S SM_VARIANTS=-1,7 timeout -k 10 200 python -u tools/probes/small_m.py >> gpurun_out/r03o_split.log 2>&1 || exit 1
done
grep -v amdgpu.ids gpurun_out/r03o_split.log
