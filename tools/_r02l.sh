mkdir -p gpurun_out
timeout -k 10 800 python -u -m comfy_gen_server_amd.tools.ab_bench --cfg "base:" --cfg "noskip:CGS_SKIPCAT=0" --cfg "nograph:CGS_GRAPHS=0" --rounds 2 > gpurun_out/r02l_ab.log 2>&1
