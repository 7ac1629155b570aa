set -o pipefail
mkdir -p gpurun_out/pmc
export TMPDIR=/tmp
P="python3 -m comfy_gen_server_amd.tools.gemm_probe gemm 16384 3840 1280"
for v in 7 5; do
  timeout -s KILL 90 rocprofv3 --kernel-trace --stats --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_LDS SQ_INSTS_VALU_MFMA_MOPS_BF16 SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE -d gpurun_out/pmc/a_v$v -o run -- $P $v 8 10 > gpurun_out/pmc/a_v$v.log 2>&1 || exit $?
  timeout -s KILL 90 rocprofv3 --kernel-trace --stats --pmc TCC_HIT_sum TCC_MISS_sum SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE -d gpurun_out/pmc/b_v$v -o run -- $P $v 8 10 > gpurun_out/pmc/b_v$v.log 2>&1 || exit $?
done
