"""Stable Cascade Stage C GEMM shapes (batch 1 with CFG: M = 2 x 576 = 1152 tokens; batch 4: 4608): every
HIP variant in TF/s (median of 3 x 10 launches), v7s = v7 with the split-K workspace."""
import math
import os
import sys

import torch

sys.path.insert(0, os.getcwd())
from comfy_gen_server_amd import _native  # noqa: E402
from comfy_gen_server_amd.ops import core  # noqa: E402

lib = _native.load_kernels()
dev = torch.device("cuda", 0)
SHAPES = [(1152, 8192, 2048, 1), (1152, 2048, 8192, 3), (1152, 6144, 2048, 1), (1152, 2048, 2048, 3),
          (4608, 2048, 8192, 3), (4608, 2048, 2048, 3),
          # SDXL batch 1 (CFG 2): level 2 M = 2048, level 1 M = 8192
          (2048, 1280, 5120, 3), (2048, 1280, 1280, 3), (2048, 10240, 1280, 1), (2048, 3840, 1280, 1),
          (8192, 640, 2560, 3), (8192, 640, 640, 3)]
for M, N, K, epi in SHAPES:
    a = torch.randn(M, K, device=dev).to(torch.bfloat16)
    w = (torch.randn(N, K, device=dev) / math.sqrt(K)).to(torch.bfloat16)
    b = torch.randn(N, device=dev).to(torch.bfloat16)
    r = torch.randn(M, N, device=dev).to(torch.bfloat16) if epi & 2 else None
    out = torch.empty(M, N, device=dev, dtype=torch.bfloat16)
    ws = core._v7_ws(M, N, K, dev)
    res = {}
    # (split-K variants of the small-tile kernels were measured here and removed: profiles/r03/splitk_small_tile.log)
    for name, v in [("v6", 6), ("v7s", 77), ("v8", 8), ("v10", 10), ("v11", 11), ("v14", 14)]:
        def run(v=v):
            if v == 77:
                if ws is None:
                    return -1
                return lib.cgs_gemm_bf16_v7ws(a.data_ptr(), w.data_ptr(), out.data_ptr(), b.data_ptr(),
                                              None if r is None else r.data_ptr(), M, N, K, K, K, N, N if r is not None else 0,
                                              epi, 1.0, ws.data_ptr(), ws.numel(), core._stream())
            return lib.cgs_gemm_bf16_v(a.data_ptr(), w.data_ptr(), out.data_ptr(), b.data_ptr(),
                                       None if r is None else r.data_ptr(), M, N, K, K, K, N, N if r is not None else 0,
                                       epi, 1.0, v, core._stream())
        if run() != 0:
            res[name] = 0
            continue
        ts = []
        for _ in range(3):
            torch.cuda.synchronize()
            s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            s.record()
            for _ in range(10):
                run()
            e.record()
            torch.cuda.synchronize()
            ts.append(s.elapsed_time(e) / 10)
        res[name] = 2.0 * M * N * K / sorted(ts)[1] / 1e9
    print(f"M={M} N={N} K={K} epi={epi} ws={'yes' if ws is not None else 'no'}: " +
          " ".join(f"{k}={v:.0f}" for k, v in res.items()), flush=True)
    del a, w, out, r, ws
