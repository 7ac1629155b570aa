"""In-process interleaved A/B (same data, same box):
  1. v6 (256x160) DMA placement modes (cgs_v6_set_mode 0/1/2) on the SDXL N = 640 / 1280 GEMMs and the
     Cout = 320 / 640 convs that run on v6;
  2. column-split hybrid for the 1.25-round GEMMs (M = 16384, N = 1280): v7 on columns [0, 1024)
     (exactly one round of 256x256 tiles) + a small-tile kernel on [1024, 1280), vs v6 / v7 split-K whole.
Prints TF/s (median of 3 rounds) and the rel. error vs an fp32 reference of one row block."""
import math
import os
import sys

import torch

sys.path.insert(0, os.getcwd())
from comfy_gen_server_amd import _native  # noqa: E402
from comfy_gen_server_amd.ops import core  # noqa: E402

lib = _native.load_kernels()
dev = torch.device("cuda", 0)
MODES = [int(m) for m in os.environ.get("V6_MODES", "0,1,3").split(",")]


def timeit(fn, iters=20):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(iters):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / iters


def ab(name, flops, runs, check):
    """runs: {label: (setup, fn)}; 3 interleaved rounds."""
    res = {k: [] for k in runs}
    for _ in range(3):
        for k, (setup, fn) in runs.items():
            setup()
            res[k].append(timeit(fn))
    errs = {}
    for k, (setup, fn) in runs.items():
        setup()
        fn()
        torch.cuda.synchronize()
        errs[k] = check()
    lib.cgs_v6_set_mode(0)
    line = " ".join(f"{k}={flops / sorted(v)[1] / 1e9:.0f}({errs[k]:.1e})" for k, v in res.items())
    print(f"{name:24s} {line}", flush=True)


GEMMS = [("out1280+res", 16384, 1280, 1280, True), ("proj1280", 16384, 1280, 1280, False),
         ("ffout1280+res", 16384, 1280, 5120, True), ("out640+res", 65536, 640, 640, True),
         ("ffout640+res", 65536, 640, 2560, True)]
for name, M, N, K, res in GEMMS:
    a = torch.randn(M, K, device=dev).to(torch.bfloat16)
    w = (torch.randn(N, K, device=dev) / math.sqrt(K)).to(torch.bfloat16)
    b = torch.randn(N, device=dev).to(torch.bfloat16)
    r = torch.randn(M, N, device=dev).to(torch.bfloat16) if res else None
    out = torch.empty(M, N, device=dev, dtype=torch.bfloat16)
    epi = core.EPI_BIAS | (core.EPI_RESIDUAL if res else 0)
    ref = a[:512].float() @ w.float().t() + b.float() + (r[:512].float() if res else 0)
    ws = core._v7_ws(M, N, K, dev)

    def check():
        return ((out[:512].float() - ref).norm() / ref.norm()).item()

    def v(variant, n0=0, n1=N, ws=None):
        rp = None if r is None else r.data_ptr() + 2 * n0
        if ws is not None:
            return lib.cgs_gemm_bf16_v7ws(a.data_ptr(), w.data_ptr() + 2 * n0 * K, out.data_ptr() + 2 * n0,
                                          b.data_ptr() + 2 * n0, rp, M, n1 - n0, K, K, K, N, N if res else 0, epi, 1.0,
                                          ws.data_ptr(), ws.numel(), core._stream())
        return lib.cgs_gemm_bf16_v(a.data_ptr(), w.data_ptr() + 2 * n0 * K, out.data_ptr() + 2 * n0,
                                   b.data_ptr() + 2 * n0, rp, M, n1 - n0, K, K, K, N, N if res else 0, epi, 1.0,
                                   variant, core._stream())

    runs = {f"v6ds{m}": ((lambda m=m: lib.cgs_v6_set_mode(m)), (lambda: v(6))) for m in MODES}
    runs["v7ws"] = ((lambda: None), (lambda: v(7, ws=ws)))
    if N == 1280 and os.environ.get("HYBRID"):
        for tv in (8, 10, 11, 14):
            runs[f"v7+t{tv}"] = ((lambda: None), (lambda tv=tv: (v(7, 0, 1024), v(tv, 1024, N))))
    ab(name, 2.0 * M * N * K, runs, check)
    del a, w, b, r, out, ws

CONVS = [("L0 res 320", 16, 128, 128, 320, 320, 3, 1), ("L0 out-res 960->320", 16, 128, 128, 960, 320, 3, 1),
         ("L0 down s2", 16, 128, 128, 320, 320, 3, 2), ("skip 1x1 960->320", 16, 128, 128, 960, 320, 1, 1),
         ("L1 res 320->640", 16, 64, 64, 320, 640, 3, 1)]
for name, N, H, W, Cin, Cout, k, s in CONVS:
    p = k // 2
    x = (torch.rand(N, H, W, Cin, device=dev) * 2 - 1).to(torch.bfloat16)
    w = ((torch.rand(Cout, k, k, Cin, device=dev) * 2 - 1) / math.sqrt(Cin * k * k)).to(torch.bfloat16)
    b = torch.zeros(Cout, device=dev, dtype=torch.bfloat16)
    Ho, Wo = (H + 2 * p - k) // s + 1, (W + 2 * p - k) // s + 1
    out = torch.empty(N, Ho, Wo, Cout, device=dev, dtype=torch.bfloat16)
    ref = torch.nn.functional.conv2d(x[:1].permute(0, 3, 1, 2).float(), w.permute(0, 3, 1, 2).float(), None, s, p)
    ref = ref.permute(0, 2, 3, 1)

    def check():
        return ((out[:1].float() - ref).norm() / ref.norm()).item()

    def cv(variant):
        return lib.cgs_conv2d_nhwc_v(x.data_ptr(), None, Cin, w.data_ptr(), b.data_ptr(), None, out.data_ptr(), N, H, W,
                                     Cin, Cout, k, k, s, p, Ho, Wo, 0, variant, core._stream())

    CMODES = [int(m) for m in os.environ.get("V6_CONV_MODES", ",".join(map(str, MODES))).split(",")]
    runs = {f"v6ds{m}": ((lambda m=m: lib.cgs_v6_set_mode(m)), (lambda: cv(6))) for m in CMODES}
    runs["v5"] = ((lambda: None), (lambda: cv(5)))
    ab(name, 2.0 * N * Ho * Wo * Cout * Cin * k * k, runs, check)
    del x, w, out
