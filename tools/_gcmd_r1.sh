export CGS_AUTOTUNE=0
rocprofv3 --list-avail > gpurun_out/counters.txt 2>&1 || true
tools/gpu_steps.sh \
  "300|pmc_v6a|rocprofv3 --kernel-trace --stats --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_LDS SQ_INSTS_VALU_MFMA_MOPS_BF16 -d gpurun_out/pmc_v6a -o run -- python -m comfy_gen_server_amd.tools.gemm_probe gemm 4096 4096 4096 6 8 10" \
  "300|pmc_v6b|rocprofv3 --kernel-trace --stats --pmc TCC_HIT_sum TCC_MISS_sum SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE -d gpurun_out/pmc_v6b -o run -- python -m comfy_gen_server_amd.tools.gemm_probe gemm 4096 4096 4096 6 8 10" \
  "300|pmc_v5a|rocprofv3 --kernel-trace --stats --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_LDS SQ_INSTS_VALU_MFMA_MOPS_BF16 -d gpurun_out/pmc_v5a -o run -- python -m comfy_gen_server_amd.tools.gemm_probe gemm 4096 4096 4096 5 8 10" \
  "300|pmc_v5b|rocprofv3 --kernel-trace --stats --pmc TCC_HIT_sum TCC_MISS_sum SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE -d gpurun_out/pmc_v5b -o run -- python -m comfy_gen_server_amd.tools.gemm_probe gemm 4096 4096 4096 5 8 10"
