"""fp32 path timings (csrc/kernels/f32.hip) against the vendor libraries through ATen on the same box:
GEMM (hipBLASLt fp32), 3x3 conv (MIOpen fp32) and the SDXL VAE decode at 1024^2 in fp32 (the
--fp32-vae configuration; the ``torch_reference`` form = ATen / MIOpen ops of the same model).

    python -m comfy_gen_server_amd.tools.f32_bench
"""
from __future__ import annotations

import json

import torch
import torch.nn.functional as F


def _time(fn, iters=10, warm=3):
    for _ in range(warm):
        fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(iters):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / iters


def main():
    from .. import ops
    from ..models.layers import init_random_fast_
    from ..ops.dispatch import torch_reference
    from ..runtime.sd import VAE
    dev = torch.device("cuda")
    out = {}
    for (M, N, K) in [(4096, 4096, 4096), (16384, 1280, 1280), (8192, 512, 512)]:
        a = torch.randn(M, K, device=dev)
        w = torch.randn(N, K, device=dev)
        t_hip = _time(lambda: ops.linear(a, w))
        t_lib = _time(lambda: F.linear(a, w))
        fl = 2.0 * M * N * K
        out[f"gemm {M}x{N}x{K}"] = {"hip_tflops": round(fl / t_hip / 1e9, 1), "hipblaslt_tflops": round(fl / t_lib / 1e9, 1)}
        print(json.dumps({f"gemm {M}x{N}x{K}": out[f"gemm {M}x{N}x{K}"]}), flush=True)
    for (C, H) in [(128, 1024), (256, 512), (512, 256)]:
        x = torch.randn(1, C, H, H, device=dev).contiguous(memory_format=torch.channels_last)
        w = torch.randn(C, C, 3, 3, device=dev) * 0.02
        wn = w.permute(0, 2, 3, 1).contiguous()
        b = torch.randn(C, device=dev)
        t_hip = _time(lambda: ops.conv2d(x, w, b, 1, 1, weight_nhwc=wn))
        t_lib = _time(lambda: F.conv2d(x, w, b, 1, 1))
        fl = 2.0 * H * H * C * C * 9
        key = f"conv3x3 C={C} {H}x{H}"
        out[key] = {"hip_tflops": round(fl / t_hip / 1e9, 1), "miopen_tflops": round(fl / t_lib / 1e9, 1)}
        print(json.dumps({key: out[key]}), flush=True)
    vae = VAE(sd=None, device=dev, dtype=torch.float32)
    m = vae.first_stage_model.to(dev)
    init_random_fast_(m, seed=1)
    z = torch.randn(1, 4, 128, 128, device=dev)
    with torch.inference_mode():
        ops.reset_stats()
        t_hip = _time(lambda: m.decode(z), iters=3, warm=1)
        lib = {str(k): v for k, v in ops.stats().items() if k[1] == "lib"}
        with torch_reference():
            t_ref = _time(lambda: m.decode(z), iters=3, warm=1)
    out["vae_decode_fp32_1024"] = {"hip_ms": round(t_hip, 1), "aten_miopen_ms": round(t_ref, 1), "lib_calls": lib}
    print(json.dumps({"vae_decode_fp32_1024": out["vae_decode_fp32_1024"]}), flush=True)


if __name__ == "__main__":
    main()
