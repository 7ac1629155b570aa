"""Timing probe of the v7 split-K tail on the level-2 1280-wide shapes (see mfma_ppk.h).

python -m comfy_gen_server_amd.tools.split_probe   (CGS_V7_SPLIT_DBG selects the probe variant)
"""
from __future__ import annotations

import math
import os

import torch


def main():
    from comfy_gen_server_amd import _native
    from comfy_gen_server_amd.ops import core
    lib = _native.load_kernels()
    dev = torch.device("cuda", 0)
    dbg = os.environ.get("CGS_V7_SPLIT_DBG", "0")
    for M, N, K in [(16384, 1280, 1280), (16384, 1280, 5120), (1232, 2560, 2048), (16384, 1280, 640)]:
        a = torch.randn(M, K, device=dev).to(torch.bfloat16)
        w = (torch.randn(N, K, device=dev) / math.sqrt(K)).to(torch.bfloat16)
        out = torch.empty(M, N, device=dev, dtype=torch.bfloat16)
        nws = lib.cgs_v7_ws_bytes(M, N, K)
        ws = torch.zeros(max(nws, 1), dtype=torch.uint8, device=dev)
        res = {}
        for name, fn in [("v7", lambda: lib.cgs_gemm_bf16_v(a.data_ptr(), w.data_ptr(), out.data_ptr(), None, None, M,
                                                          N, K, K, K, N, 0, 0, 1.0, 7, core._stream())),
                         ("v7s", lambda: lib.cgs_gemm_bf16_v7ws(a.data_ptr(), w.data_ptr(), out.data_ptr(), None,
                                                              None, M, N, K, K, K, N, 0, 0, 1.0, ws.data_ptr(), nws,
                                                              core._stream()))]:
            for _ in range(3):
                fn()
            torch.cuda.synchronize()
            s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            it = 50
            s.record()
            for _ in range(it):
                fn()
            e.record()
            torch.cuda.synchronize()
            res[name] = s.elapsed_time(e) / it * 1000
        print(f"dbg={dbg} M={M} N={N} K={K} ws={nws} v7={res['v7']:.1f}us v7s={res['v7s']:.1f}us", flush=True)


if __name__ == "__main__":
    main()
