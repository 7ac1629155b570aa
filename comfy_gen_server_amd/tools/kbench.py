"""Kernel micro-benchmarks on the SDXL shapes of SURVEY Appendix A (B=16 UNet batch = 8 images x CFG).

Compares the hand-written HIP kernels with the vendor library path through ATen (hipBLASLt GEMM,
MIOpen conv, SDPA attention) in one process, interleaved (cdna guide §5.4 rule 24), on random data.
Usage: python -m comfy_gen_server_amd.tools.kbench [--quick]
"""
from __future__ import annotations

import json
import math
import sys
import time

import torch
import torch.nn.functional as F


def _time(fn, iters=20, warm=3):
    for _ in range(warm):
        fn()
    torch.cuda.synchronize()
    ts = []
    for _ in range(iters):
        s = torch.cuda.Event(enable_timing=True)
        e = torch.cuda.Event(enable_timing=True)
        s.record()
        fn()
        e.record()
        torch.cuda.synchronize()
        ts.append(s.elapsed_time(e))
    ts.sort()
    return ts[len(ts) // 2]


def main(quick=False, attn_only=False, gemm_only=False):
    import os
    os.environ["CGS_AUTOTUNE"] = "0"      # explicit variants below; the per-shape tuner would override them
    from comfy_gen_server_amd import ops
    from comfy_gen_server_amd.ops import core
    from comfy_gen_server_amd.ops.dispatch import set_backend_override
    dev = torch.device("cuda", 0)
    torch.manual_seed(0)
    res = {"gemm": [], "attention": [], "groupnorm": [], "layernorm": [], "conv": []}
    B = 16
    gemm_shapes = [(B * 1024, 1280, 1280), (B * 1024, 1280, 3840), (B * 1024, 10240, 1280), (B * 1024, 1280, 5120),
                   (B * 4096, 640, 640), (B * 4096, 5120, 640), (B * 4096, 640, 2560), (B * 77, 1280, 2048)]
    if quick:
        gemm_shapes = gemm_shapes[:3]
    if attn_only:
        gemm_shapes = []
    if gemm_only:
        gemm_shapes = [(4096, 4096, 4096), (8192, 8192, 8192)] + gemm_shapes[:-1]
    for M, N, K in gemm_shapes:
        a = torch.randn(M, K, device=dev).to(torch.bfloat16)
        w = (torch.randn(N, K, device=dev) / math.sqrt(K)).to(torch.bfloat16)
        bias = torch.randn(N, device=dev).to(torch.bfloat16)
        fl = 2.0 * M * N * K
        lib = ops.dispatch._native.load_kernels()
        ent = dict(M=M, N=N, K=K)
        for var in (3, 4, 5, 6):
            lib.cgs_gemm_set_variant(var)
            for g in ((1, 8) if var >= 3 else (8,)):
                lib.cgs_set_tile_group(g)
                t = _time(lambda: ops.linear(a, w, bias))
                ent[f"v{var}g{g}_tflops"] = fl / t / 1e9
        lib.cgs_set_tile_group(8)
        lib.cgs_gemm_set_variant(-1)
        t_lib = _time(lambda: F.linear(a, w, bias))
        ent["lib_tflops"] = fl / t_lib / 1e9
        res["gemm"].append(ent)
        if gemm_only:
            print(json.dumps({k: (round(v) if isinstance(v, float) else v) for k, v in ent.items()}), flush=True)
    if gemm_only:
        return res
    att_shapes = [(B, 20, 1024, 1024, 64), (B, 10, 4096, 4096, 64), (B, 20, 1024, 77, 64), (B, 10, 4096, 77, 64)]
    if quick:
        att_shapes = att_shapes[:2]
    for b, h, sq, sk, d in att_shapes:
        q = torch.randn(b, sq, h * d, device=dev).to(torch.bfloat16)
        k = torch.randn(b, sk, h * d, device=dev).to(torch.bfloat16)
        v = torch.randn(b, sk, h * d, device=dev).to(torch.bfloat16)
        fl = 4.0 * b * h * sq * sk * d
        lib = ops.dispatch._native.load_kernels()
        ent = dict(B=b, H=h, Sq=sq, Sk=sk, D=d)
        ref = None
        for var, name in ((1, "generic"), (2, "d64"), (5, "d64q128"), (0, "auto")):
            lib.cgs_attn_set_variant(var)
            y = ops.attention(q, k, v, h).float()
            if ref is None:
                ref = y
            ent[f"{name}_maxdiff"] = (y - ref).abs().max().item()
            t_hip = _time(lambda: ops.attention(q, k, v, h))
            ent[f"{name}_ms"] = t_hip
            ent[f"{name}_tflops"] = fl / t_hip / 1e9
        lib.cgs_attn_set_variant(0)
        qh, kh, vh = (t.view(b, -1, h, d).transpose(1, 2) for t in (q, k, v))
        t_sdpa = _time(lambda: F.scaled_dot_product_attention(qh, kh, vh))
        ent.update(sdpa_ms=t_sdpa, sdpa_tflops=fl / t_sdpa / 1e9)
        if sq == sk:   # q/k/v as views of one fused QKV projection (the UNet's layout)
            qkv = torch.randn(b, sq, 3 * h * d, device=dev).to(torch.bfloat16)
            qv, kv_, vv = qkv.split(h * d, dim=-1)
            t_f = _time(lambda: ops.attention(qv, kv_, vv, h))
            ent.update(fused_qkv_ms=t_f, fused_qkv_tflops=fl / t_f / 1e9)
        res["attention"].append(ent)
        if attn_only:
            print(json.dumps(ent), flush=True)
    if attn_only:
        return res
    for N, C, H, W in [(B, 320, 128, 128), (B, 640, 64, 64), (B, 1280, 32, 32)]:
        x = torch.randn(N, C, H, W, device=dev).to(torch.bfloat16).contiguous(memory_format=torch.channels_last)
        wt = torch.randn(C, device=dev).to(torch.bfloat16)
        bt = torch.randn(C, device=dev).to(torch.bfloat16)
        nbytes = 2 * x.numel() * 2
        t_hip = _time(lambda: ops.group_norm(x, 32, wt, bt, 1e-5, silu=True))
        t_lib = _time(lambda: F.silu(F.group_norm(x, 32, wt, bt, 1e-5)))
        res["groupnorm"].append(dict(shape=[N, C, H, W], hip_ms=t_hip, lib_ms=t_lib, hip_GBps=nbytes / t_hip / 1e6,
                                     lib_GBps=nbytes / t_lib / 1e6))
    for rows, C in [(B * 4096, 640), (B * 1024, 1280)]:
        x = torch.randn(rows, C, device=dev).to(torch.bfloat16)
        wt = torch.randn(C, device=dev).to(torch.bfloat16)
        bt = torch.randn(C, device=dev).to(torch.bfloat16)
        nbytes = 2 * x.numel() * 2
        t_hip = _time(lambda: ops.layer_norm(x, wt, bt))
        t_lib = _time(lambda: F.layer_norm(x, (C,), wt, bt))
        res["layernorm"].append(dict(rows=rows, C=C, hip_ms=t_hip, lib_ms=t_lib, hip_GBps=nbytes / t_hip / 1e6,
                                     lib_GBps=nbytes / t_lib / 1e6))
    for N, Ci, H, W, Co in [(B, 320, 128, 128, 320), (B, 640, 128, 128, 320), (B, 960, 128, 128, 320),
                            (B, 640, 64, 64, 640), (B, 1280, 32, 32, 1280),
                            (B, 1920, 32, 32, 1280), (1, 256, 512, 512, 256), (1, 128, 1024, 1024, 128)]:
        x = torch.randn(N, Ci, H, W, device=dev).to(torch.bfloat16).contiguous(memory_format=torch.channels_last)
        wt = (torch.randn(Co, Ci, 3, 3, device=dev) / math.sqrt(Ci * 9)).to(torch.bfloat16)
        bt = torch.randn(Co, device=dev).to(torch.bfloat16)
        fl = 2.0 * N * H * W * Co * Ci * 9
        t_lib = _time(lambda: F.conv2d(x, wt, bt, 1, 1))
        entry = dict(shape=[N, Ci, H, W, Co], lib_ms=t_lib, lib_tflops=fl / t_lib / 1e9)
        if ops.dispatch._native.has_kernel("cgs_conv2d_nhwc"):
            wn = wt.permute(0, 2, 3, 1).contiguous()
            set_backend_override("conv", "hip")
            lib = ops.dispatch._native.load_kernels()
            for var in (2, 3, 4, 5, 6):
                lib.cgs_conv_set_variant(var)
                for g in (8,):
                    lib.cgs_conv_set_tile_group(g)
                    t_hip = _time(lambda: ops.conv2d(x, wt, bt, 1, 1, weight_nhwc=wn))
                    entry.update({f"v{var}g{g}_tflops": fl / t_hip / 1e9})
            lib.cgs_conv_set_tile_group(8)
            lib.cgs_conv_set_variant(-1)
            set_backend_override("conv", None)
        res["conv"].append(entry)
    print(json.dumps(res, indent=1))
    return res


if __name__ == "__main__":
    main(quick="--quick" in sys.argv, attn_only="--attn" in sys.argv, gemm_only="--gemm" in sys.argv)
