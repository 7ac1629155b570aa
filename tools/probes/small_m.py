"""Batch-1 SDXL GEMM shapes (M = 2 x tokens: 2048 at level 2, 8192 at level 1) on every kernel variant,
plus hipBLASLt (F.linear) as the vendor reference. Median of 3 rounds x 20 launches, TF/s."""
import math
import os
import sys

import torch
import torch.nn.functional as F

sys.path.insert(0, os.getcwd())
from comfy_gen_server_amd import _native  # noqa: E402
from comfy_gen_server_amd.ops import core  # noqa: E402

# name, M, N, K, geglu, residual, lnfold
SHAPES = [("L2 qkv(ln)", 2048, 3840, 1280, False, False, True), ("L2 q(ln)", 2048, 1280, 1280, False, False, True),
          ("L2 out+res", 2048, 1280, 1280, False, True, False), ("L2 geglu(ln)", 2048, 10240, 1280, True, False, True),
          ("L2 ffout+res", 2048, 1280, 5120, False, True, False), ("L2 proj", 2048, 1280, 1280, False, False, False),
          ("L1 qkv(ln)", 8192, 1920, 640, False, False, True), ("L1 out+res", 8192, 640, 640, False, True, False),
          ("L1 geglu(ln)", 8192, 5120, 640, True, False, True), ("L1 ffout+res", 8192, 640, 2560, False, True, False),
          ("C 2048->8192", 1152, 8192, 2048, False, False, False), ("C 8192->2048+res", 1152, 2048, 8192, False, True, False)]
VARIANTS = [int(v) for v in os.environ.get("SM_VARIANTS", "-1,6,7,8,10,11,12,13,14").split(",")]
lib = _native.load_kernels()
dev = torch.device("cuda", 0)


def timeit(fn):
    ts = []
    for _ in range(3):
        fn()
        torch.cuda.synchronize()
        s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        s.record()
        for _ in range(20):
            fn()
        e.record()
        torch.cuda.synchronize()
        ts.append(s.elapsed_time(e) / 20)
    return sorted(ts)[1]


for name, M, N, K, gg, res, ln in SHAPES:
    a = torch.randn(M, K, device=dev).to(torch.bfloat16)
    w = (torch.randn(N, K, device=dev) / math.sqrt(K)).to(torch.bfloat16)
    b = torch.randn(N, device=dev).to(torch.bfloat16)
    nout = N // 2 if gg else N
    r = torch.randn(M, nout, device=dev).to(torch.bfloat16) if res else None
    out = torch.empty(M, nout, device=dev, dtype=torch.bfloat16)
    epi = core.EPI_BIAS | (core.EPI_GEGLU if gg else 0) | (core.EPI_RESIDUAL if res else 0)
    rs = core.layernorm_stats(a, 1e-5) if ln else None
    cs = w.float().sum(dim=1).contiguous() if ln else None
    flops = 2 * M * N * K
    cols = []
    for v in VARIANTS:
        if ln:
            if v not in (-1, 8, 10, 11, 12, 13, 14):
                continue
            ws = core._v7_ws(M, N, K, dev) if v == -1 else None

            def run(v=v, ws=ws):
                return lib.cgs_gemm_bf16_lnfold_v(a.data_ptr(), w.data_ptr(), out.data_ptr(), b.data_ptr(),
                                                  rs.data_ptr(), cs.data_ptr(), M, N, K, K, K, nout, epi,
                                                  None if ws is None else ws.data_ptr(),
                                                  0 if ws is None else ws.numel(), v, core._stream())
        else:
            if v == -1:
                continue
            ws = core._v7_ws(M, N, K, dev) if v == 7 else None

            def run(v=v, ws=ws):
                if ws is not None:
                    return lib.cgs_gemm_bf16_v7ws(a.data_ptr(), w.data_ptr(), out.data_ptr(), b.data_ptr(),
                                                  None if r is None else r.data_ptr(), M, N, K, K, K, nout,
                                                  nout if res else 0, epi, 1.0, ws.data_ptr(), ws.numel(),
                                                  core._stream())
                return lib.cgs_gemm_bf16_v(a.data_ptr(), w.data_ptr(), out.data_ptr(), b.data_ptr(),
                                           None if r is None else r.data_ptr(), M, N, K, K, K, nout,
                                           nout if res else 0, epi, 1.0, v, core._stream())
        rc = run()
        if rc != 0:
            cols.append(f"v{v}=n/a")
            continue
        cols.append(f"v{v if v >= 0 else 'def'}={flops / timeit(run) / 1e9:.0f}")
    if not gg:
        t = timeit(lambda: F.linear(a, w, b) if r is None else torch.addmm(r, a, w.t()))
        cols.append(f"lib={flops / t / 1e9:.0f}")
    print(f"{name:18s} M={M} N={N} K={K} TF/s: " + " ".join(cols), flush=True)
