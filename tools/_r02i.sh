mkdir -p gpurun_out
timeout -k 10 500 python -u -m comfy_gen_server_amd.tools.conv_table gpurun_out/r02i_conv_table.md --vae > gpurun_out/r02i_conv.log 2>&1
