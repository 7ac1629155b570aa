"""SDXL batch-1 LayerNorm-folded GEMM shapes (M = 2048 level 2, 8192 level 1) on every candidate."""
import math
import os
import sys

import torch

sys.path.insert(0, os.getcwd())
from comfy_gen_server_amd import _native  # noqa: E402
from comfy_gen_server_amd.ops import core  # noqa: E402

lib = _native.load_kernels()
dev = torch.device("cuda", 0)
for M, N, K in [(2048, 3840, 1280), (2048, 1280, 1280), (8192, 1920, 640), (8192, 640, 640)]:
    a = torch.randn(M, K, device=dev).to(torch.bfloat16)
    w = (torch.randn(N, K, device=dev) / math.sqrt(K)).to(torch.bfloat16)
    b = torch.randn(N, device=dev).to(torch.bfloat16)
    rs = core.layernorm_stats(a, 1e-5)
    cs = w.float().sum(dim=1).contiguous()
    out = torch.empty(M, N, device=dev, dtype=torch.bfloat16)
    ws = core._v7_ws(M, N, K, dev)
    res = {}
    for v in (6, 7, 8, 10, 11, 12, 13, 14):
        def run(v=v):
            use_ws = ws is not None and v == 7
            return lib.cgs_gemm_bf16_lnfold_v(a.data_ptr(), w.data_ptr(), out.data_ptr(), b.data_ptr(), rs.data_ptr(),
                                              cs.data_ptr(), M, N, K, K, K, N, core.EPI_BIAS,
                                              ws.data_ptr() if use_ws else None, ws.numel() if use_ws else 0, v,
                                              core._stream())
        if run() != 0:
            continue
        ts = []
        for _ in range(3):
            torch.cuda.synchronize()
            s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            s.record()
            for _ in range(20):
                run()
            e.record()
            torch.cuda.synchronize()
            ts.append(s.elapsed_time(e) / 20)
        res[v] = sorted(ts)[1]
    print(f"ln M={M} N={N} K={K}: " + " ".join(f"v{v}={2 * M * N * K / t / 1e9:.0f}({t * 1e3:.0f}us)" for v, t in res.items()),
          flush=True)
    del a, w, out, ws
