#!/bin/bash
# round-3 probe 16: which hipBLASLt kernels serve the small-M shapes (names, grid, workgroup)
cd "${GRAFT_REPO_ROOT:-.}" || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp
LIB_SHAPES=small timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/r03p -o run -- python3 tools/probes/lib_gemm_names.py > gpurun_out/r03p_lib.log 2>&1 || exit 1
cp /tmp/r03p/run_kernel_stats.csv gpurun_out/r03p_lib_kernel_stats.csv
python3 - <<'PY' > gpurun_out/r03p_lib_dispatch.txt
import csv, collections
rows = list(csv.DictReader(open('/tmp/r03p/run_kernel_trace.csv')))
seen = collections.OrderedDict()
for r in rows:
    n = r.get('Kernel_Name', '')
    if 'Cijk' not in n:
        continue
    k = (n[:160], r.get('Grid_Size_X', r.get('Grid_Size', '')), r.get('Workgroup_Size_X', r.get('Workgroup_Size', '')), r.get('LDS_Block_Size', r.get('Lds_Size', '')))
    seen[k] = seen.get(k, 0) + 1
for k, v in seen.items():
    print(v, k)
print(list(rows[0].keys()) if rows else 'no rows')
PY
grep -v amdgpu.ids gpurun_out/r03p_lib.log | grep "M=" ; cat gpurun_out/r03p_lib_dispatch.txt
