#!/bin/bash
# round-3 probe 27: PMC anatomy of v6 (split DMAs) vs v7 on a short-K and a long-K SDXL shape
cd "${GRAFT_REPO_ROOT:-.}" || exit 1
mkdir -p gpurun_out/pmc
export TMPDIR=/tmp HSA_ENABLE_IPC_MODE_LEGACY=0
A="SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_INST_LDS GRBM_GUI_ACTIVE"
B="SQ_ACTIVE_INST_VMEM SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_SCA SQ_INSTS_VMEM SQ_INSTS_LDS SQ_INSTS_VALU SQ_INSTS_SALU"
for shp in "16384 3840 1280" "16384 1280 5120"; do
  for v in 6 7; do
    t=$(echo $shp | tr ' ' x)_v$v
    for pass in A B; do
      eval C=\$$pass
      timeout -s KILL 60 rocprofv3 --kernel-trace --pmc $C -d /tmp/pmc_${t}_$pass -o run -- python3 -m comfy_gen_server_amd.tools.gemm_probe gemm $shp $v 8 10 > gpurun_out/pmc/${t}_$pass.log 2>&1 || { echo "pmc $t $pass failed"; tail -5 gpurun_out/pmc/${t}_$pass.log; exit 1; }
      db=$(find /tmp/pmc_${t}_$pass -name "*results.db" | head -n1)
      echo "### $t pass $pass"; python -m comfy_gen_server_amd.tools.pmc_summary gemm_bf16 "$db"
    done
  done
done
