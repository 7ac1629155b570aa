"""In-process interleaved A/B of v7 epilogue variants (cgs_v7_set_dbg bits), same data, same box."""
import math
import os
import sys

import torch

sys.path.insert(0, os.getcwd())
from comfy_gen_server_amd import _native  # noqa: E402
from comfy_gen_server_amd.ops import core  # noqa: E402

SHAPES = [("qkv1280", 16384, 3840, 1280, False, False), ("geglu1280", 16384, 10240, 1280, True, False),
          ("geglu640", 65536, 5120, 640, True, False), ("qkv640", 65536, 1920, 640, False, False),
          ("out1280+res", 16384, 1280, 1280, False, True), ("ffout640+res", 65536, 640, 2560, False, True),
          ("k5120", 16384, 4096, 5120, False, False),
          # the production forms: LayerNorm folded in (qkv / GEGLU of every transformer block)
          ("ln:qkv1280", 16384, 3840, 1280, False, False), ("ln:geglu1280", 16384, 10240, 1280, True, False),
          ("ln:qkv640", 65536, 1920, 640, False, False), ("ln:geglu640", 65536, 5120, 640, True, False)]
VARIANTS = [int(v) for v in os.environ.get("AB_VARIANTS", "0,32,8,40").split(",")]
lib = _native.load_kernels()
dev = torch.device("cuda", 0)
for name, M, N, K, gg, res in SHAPES:
    a = torch.randn(M, K, device=dev).to(torch.bfloat16)
    w = (torch.randn(N, K, device=dev) / math.sqrt(K)).to(torch.bfloat16)
    b = torch.randn(N, device=dev).to(torch.bfloat16)
    nout = N // 2 if gg else N
    r = torch.randn(M, nout, device=dev).to(torch.bfloat16) if res else None
    out = torch.empty(M, nout, device=dev, dtype=torch.bfloat16)
    epi = core.EPI_BIAS | (core.EPI_GEGLU if gg else 0) | (core.EPI_RESIDUAL if res else 0)

    ln = name.startswith("ln:")
    if ln:
        rs = core.layernorm_stats(a, 1e-5)
        cs = w.float().sum(dim=1).contiguous()
        ws = core._v7_ws(M, N, K, dev)

    def run():
        if ln:
            return lib.cgs_gemm_bf16_lnfold(a.data_ptr(), w.data_ptr(), out.data_ptr(), b.data_ptr(), rs.data_ptr(),
                                            cs.data_ptr(), M, N, K, K, K, nout, core.EPI_BIAS | (core.EPI_GEGLU if gg else 0),
                                            None if ws is None else ws.data_ptr(), 0 if ws is None else ws.numel(),
                                            core._stream())
        return lib.cgs_gemm_bf16_v(a.data_ptr(), w.data_ptr(), out.data_ptr(), b.data_ptr(),
                                   None if r is None else r.data_ptr(), M, N, K, K, K, nout, nout if res else 0,
                                   epi, 1.0, 7, core._stream())
    res_t = {v: [] for v in VARIANTS}
    for rnd in range(3):
        for v in VARIANTS:
            lib.cgs_v7_set_dbg(v)
            for _ in range(3):
                run()
            torch.cuda.synchronize()
            s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            s.record()
            for _ in range(20):
                run()
            e.record()
            torch.cuda.synchronize()
            res_t[v].append(s.elapsed_time(e) / 20)
    outs = {}
    for v in VARIANTS:
        lib.cgs_v7_set_dbg(v)
        out.fill_(0)
        run()
        torch.cuda.synchronize()
        outs[v] = out.clone()
    same = all(torch.equal(outs[v], outs[VARIANTS[0]]) for v in VARIANTS)
    lib.cgs_v7_set_dbg(0)
    line = " ".join(f"dbg{v}={2 * M * N * K / sorted(ts)[1] / 1e9:.0f}" for v, ts in res_t.items())
    line += f" bitwise-equal={same}"
    del outs
    print(f"{name:14s} M={M} N={N} K={K} TF/s (median of 3) {line}", flush=True)
