mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_kernels_gpu.py -x -q -k "conv" --timeout 200 --timeout-method thread > gpurun_out/r02j_tests.log 2>&1 || exit $?
timeout -k 10 400 python -u -m comfy_gen_server_amd.tools.conv_table gpurun_out/r02j_conv_table.md --vae > gpurun_out/r02j_conv.log 2>&1
