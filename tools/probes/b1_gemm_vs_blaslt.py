"""SDXL batch-1 GEMM shapes (UNet batch 2 under CFG: M = 2048 tokens at level 2, 8192 at level 1): the
dispatched HIP kernel (ops.linear, packaged tuning table) vs hipBLASLt (torch.mm), plain GEMM + bias, in one
process, interleaved; median of 5."""
import os
import statistics
import sys

import torch

sys.path.insert(0, os.getcwd())
from comfy_gen_server_amd.ops import core  # noqa: E402

dev = torch.device("cuda", 0)
SHAPES = [("out1280", 2048, 1280, 1280), ("ffout1280", 2048, 1280, 5120), ("qkv1280", 2048, 3840, 1280),
          ("geglu1280 (plain)", 2048, 10240, 1280), ("out640", 8192, 640, 640), ("ffout640", 8192, 640, 2560),
          ("qkv640", 8192, 1920, 640), ("geglu640 (plain)", 8192, 5120, 640)]


def _t(f, n=20):
    f()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(n):
        f()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / n * 1e3


for name, M, N, K in SHAPES:
    a = torch.randn(M, K, device=dev).to(torch.bfloat16)
    w = (torch.randn(N, K, device=dev) / K ** 0.5).to(torch.bfloat16)
    b = torch.randn(N, device=dev).to(torch.bfloat16)
    ours, lib = [], []
    for _ in range(5):
        ours.append(_t(lambda: core.linear(a, w, b)))
        lib.append(_t(lambda: torch.addmm(b, a, w.t())))
    o, h = statistics.median(ours), statistics.median(lib)
    fl = 2.0 * M * N * K
    print(f"{name:18s} M={M} N={N} K={K}: ours {o:6.1f} us ({fl / o / 1e6:5.0f} TF/s)  hipBLASLt {h:6.1f} us "
          f"({fl / h / 1e6:5.0f} TF/s)  ours/lib {h / o:.2f}x", flush=True)
