export CGS_AUTOTUNE=0
tools/gpu_steps.sh \
 "300|pytest_attn|python -m pytest tests/test_kernels_gpu.py -x -q -k attention" \
 "300|kbench_attn|python -m comfy_gen_server_amd.tools.kbench --attn"
