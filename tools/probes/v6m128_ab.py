"""The 128 x 160 v6 GEMM tile (variant 19) and its one-wave-group 128 x 80 form (variant 20) vs the 256 x 160 v6 (6) and the small-tile family (8 / 10 / 14) on the
SDXL batch-1 shapes (M = 2048 / 8192 tokens under CFG), plain + bias, + residual, and the LayerNorm-folded form;
one process, interleaved, median of 5; every output checked against an fp32 reference.

python tools/probes/v6m128_ab.py"""
import os
import statistics
import sys

import torch

sys.path.insert(0, os.getcwd())
from comfy_gen_server_amd.ops import core  # noqa: E402

dev = torch.device("cuda", 0)
lib = core._lib()
s = core._stream()


def _t(f, n=20):
    f()
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(n):
        f()
    b.record()
    torch.cuda.synchronize()
    return a.elapsed_time(b) / n * 1e3


torch.manual_seed(0)
for name, M, N, K, kind in [("out1280+res", 2048, 1280, 1280, "res"), ("ffout1280+res", 2048, 1280, 5120, "res"),
                            ("q1280 (LN)", 2048, 1280, 1280, "ln"), ("qkv1280 (LN)", 2048, 3840, 1280, "ln"),
                            ("out640+res", 8192, 640, 640, "res"), ("ffout640+res", 8192, 640, 2560, "res"),
                            ("q640 (LN)", 8192, 640, 640, "ln"), ("kv2560 plain", 2048, 2560, 1280, "plain"),
                            ("out1280+res b16", 16384, 1280, 1280, "res")]:
    a = torch.randn(M, K, device=dev).to(torch.bfloat16)
    w = (torch.randn(N, K, device=dev) / K ** 0.5).to(torch.bfloat16)
    b = torch.randn(N, device=dev).to(torch.bfloat16)
    r = torch.randn(M, N, device=dev).to(torch.bfloat16) if kind == "res" else None
    rs = cs = None
    if kind == "ln":
        mu = a.float().mean(1)
        rstd = torch.rsqrt(a.float().var(1, unbiased=False) + 1e-5)
        rs = torch.stack([mu, rstd], 1).contiguous()
        cs = w.float().sum(1).contiguous()
        ref = ((a.float() - mu[:, None]) * rstd[:, None]) @ w.float().t() + b.float()
    else:
        ref = a.float() @ w.float().t() + b.float() + (r.float() if r is not None else 0)
    epi = 1 | (2 if r is not None else 0)
    outs = {}

    def run(v):
        o = outs.setdefault(v, torch.empty(M, N, device=dev, dtype=torch.bfloat16))
        if kind == "ln":
            rc = lib.cgs_gemm_bf16_lnfold_v(a.data_ptr(), w.data_ptr(), o.data_ptr(), b.data_ptr(), rs.data_ptr(),
                                            cs.data_ptr(), M, N, K, K, K, N, 1, None, 0, v, s)
        else:
            rc = lib.cgs_gemm_bf16_v(a.data_ptr(), w.data_ptr(), o.data_ptr(), b.data_ptr(), core._ptr(r), M, N, K, K,
                                     K, N, N if r is not None else 0, epi, 1.0, v, s)
        assert rc == 0, (v, rc)
    vs = [6, 19, 20, 8, 14]
    ts = {v: [] for v in vs}
    for _ in range(5):
        for v in vs:
            ts[v].append(_t(lambda: run(v)))
    fl = 2.0 * M * N * K
    errs = {v: ((outs[v].float() - ref).norm() / ref.norm()).item() for v in vs}
    line = "  ".join(f"v{v} {statistics.median(t):.1f} us ({fl / statistics.median(t) / 1e6:.0f})" for v, t in ts.items())
    print(f"{name:16s} M={M} N={N} K={K}: {line}  max rel err {max(errs.values()):.1e}", flush=True)
    assert max(errs.values()) < 2e-2, errs
