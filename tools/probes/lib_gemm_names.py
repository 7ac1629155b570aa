"""Run hipBLASLt (through ATen) on the SDXL GEMM shapes so a rocprofv3 kernel trace names its kernels."""
import math
import os

import torch

SHAPES = [(65536, 1920, 640), (65536, 640, 640), (65536, 5120, 640), (65536, 640, 2560), (16384, 3840, 1280),
          (16384, 1280, 1280), (16384, 10240, 1280), (16384, 1280, 5120), (1232, 2560, 2048)]
if os.environ.get("LIB_SHAPES") == "small":     # batch-1 SDXL / Cascade Stage C shapes
    SHAPES = [(2048, 3840, 1280), (2048, 1280, 1280), (2048, 1280, 5120), (8192, 640, 2560), (1152, 8192, 2048),
              (1152, 2048, 8192)]

dev = torch.device("cuda", 0)
for M, N, K in SHAPES:
    a = torch.randn(M, K, device=dev).to(torch.bfloat16)
    w = (torch.randn(N, K, device=dev) / math.sqrt(K)).to(torch.bfloat16)
    b = torch.randn(N, device=dev).to(torch.bfloat16)
    for _ in range(5):
        torch.nn.functional.linear(a, w, b)
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(10):
        torch.nn.functional.linear(a, w, b)
    e.record()
    torch.cuda.synchronize()
    ms = s.elapsed_time(e) / 10
    print(f"M={M} N={N} K={K} {ms * 1e3:.1f} us {2 * M * N * K / ms / 1e9:.0f} TF/s", flush=True)
