"""v7 GEMM timing under CGS_V7_SPLIT_DBG probe bits (set in the environment before the first launch)."""
import math
import os
import sys

import torch

sys.path.insert(0, os.getcwd())
from comfy_gen_server_amd import _native  # noqa: E402
from comfy_gen_server_amd.ops import core  # noqa: E402

SHAPES = [("qkv1280", 16384, 3840, 1280, False), ("geglu1280", 16384, 10240, 1280, True),
          ("geglu640", 65536, 5120, 640, True), ("q640", 65536, 640, 640, False),
          ("k5120", 16384, 4096, 5120, False)]
lib = _native.load_kernels()
dev = torch.device("cuda", 0)
tag = os.environ.get("CGS_V7_SPLIT_DBG", "0")
for name, M, N, K, gg in SHAPES:
    a = torch.randn(M, K, device=dev).to(torch.bfloat16)
    w = (torch.randn(N, K, device=dev) / math.sqrt(K)).to(torch.bfloat16)
    b = torch.randn(N, device=dev).to(torch.bfloat16)
    nout = N // 2 if gg else N
    out = torch.empty(M, nout, device=dev, dtype=torch.bfloat16)
    epi = core.EPI_BIAS | (core.EPI_GEGLU if gg else 0)

    def run():
        return lib.cgs_gemm_bf16_v(a.data_ptr(), w.data_ptr(), out.data_ptr(), b.data_ptr(), None, M, N, K, K, K,
                                   nout, 0, epi, 1.0, 7, core._stream())
    for _ in range(3):
        run()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(20):
        run()
    e.record()
    torch.cuda.synchronize()
    ms = s.elapsed_time(e) / 20
    print(f"dbg={tag} {name} M={M} N={N} K={K} {ms * 1e3:.1f} us {2 * M * N * K / ms / 1e9:.0f} TF/s", flush=True)
