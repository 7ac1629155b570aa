"""Run one GEMM / conv configuration in a loop for PMC-counter profiling under rocprofv3.

python -m comfy_gen_server_amd.tools.gemm_probe gemm M N K [variant] [group] [iters]
python -m comfy_gen_server_amd.tools.gemm_probe conv N Cin H W Cout [variant] [group] [iters]
"""
import math
import sys

import torch


def main(argv):
    from comfy_gen_server_amd import ops, _native
    from comfy_gen_server_amd.ops.dispatch import set_backend_override
    lib = _native.load_kernels()
    dev = torch.device("cuda", 0)
    kind = argv[0]
    if kind == "gemm":
        M, N, K = (int(v) for v in argv[1:4])
        var = argv[4] if len(argv) > 4 else "-1"   # kernel variant number (16 / 17: w6) or "lib" (hipBLASLt)
        grp = int(argv[5]) if len(argv) > 5 else 8
        iters = int(argv[6]) if len(argv) > 6 else 20
        a = torch.randn(M, K, device=dev).to(torch.bfloat16)
        w = (torch.randn(N, K, device=dev) / math.sqrt(K)).to(torch.bfloat16)
        lib.cgs_set_tile_group(grp)
        out = torch.empty(M, N, device=dev, dtype=torch.bfloat16)
        from comfy_gen_server_amd.ops import core

        def fn():  # the kernel itself (no autotune table, no library candidate)
            if var == "lib":
                torch.mm(a, w.t(), out=out)
                return
            if True:
                err = lib.cgs_gemm_bf16_v(a.data_ptr(), w.data_ptr(), out.data_ptr(), None, None, M, N, K, K, K, N, 0,
                                          0, 1.0, int(var), core._stream())
            assert err == 0, err
        flops = 2.0 * M * N * K
    else:
        N, Ci, H, W, Co = (int(v) for v in argv[1:6])
        var = int(argv[6]) if len(argv) > 6 else -1
        grp = int(argv[7]) if len(argv) > 7 else 8
        iters = int(argv[8]) if len(argv) > 8 else 20
        x = torch.randn(N, Ci, H, W, device=dev).to(torch.bfloat16).contiguous(memory_format=torch.channels_last)
        wt = (torch.randn(Co, Ci, 3, 3, device=dev) / math.sqrt(Ci * 9)).to(torch.bfloat16)
        wn = wt.permute(0, 2, 3, 1).contiguous()
        lib.cgs_conv_set_variant(var)
        lib.cgs_conv_set_tile_group(grp)
        set_backend_override("conv", "hip")
        fn = lambda: ops.conv2d(x, wt, None, 1, 1, weight_nhwc=wn)  # noqa: E731
        flops = 2.0 * N * H * W * Co * Ci * 9
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(iters):
        fn()
    e.record()
    torch.cuda.synchronize()
    ms = s.elapsed_time(e) / iters
    print(f"{kind} {argv[1:]} {ms:.3f} ms {flops / ms / 1e9:.1f} TFLOP/s")


if __name__ == "__main__":
    main(sys.argv[1:])
