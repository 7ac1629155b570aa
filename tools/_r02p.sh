mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_graphs_gpu.py tests/test_image_kernels_gpu.py -x -q -k "controlnet or vae_out or step_graph" --timeout 200 --timeout-method thread > gpurun_out/r02p_tests.log 2>&1
echo "tests rc=$?" >> gpurun_out/r02p_tests.log
timeout -k 10 250 python -u -m comfy_gen_server_amd.tools.gemm_sweep gpurun_out/r02p_base.md --kseries > gpurun_out/r02p.log 2>&1 && timeout -k 10 250 python -u -m comfy_gen_server_amd.tools.gemm_sweep gpurun_out/r02p_stag.md --kseries --stagger >> gpurun_out/r02p.log 2>&1
