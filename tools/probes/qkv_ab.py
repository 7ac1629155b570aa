"""In-process A/B: fused-QKV (and other wide, non-GEGLU) GEMMs on v6 (256x160, whole rounds) vs v7
(256x256, split-K tail), plain and with the LayerNorm fold; the Cout = 640 convs on v5 / v6 / v7."""
import math
import os
import sys

import torch

sys.path.insert(0, os.getcwd())
from comfy_gen_server_amd import _native  # noqa: E402
from comfy_gen_server_amd.ops import core  # noqa: E402

lib = _native.load_kernels()
dev = torch.device("cuda", 0)


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
    res = {k: [] for k in runs}
    for _ in range(3):
        for k, fn in runs.items():
            res[k].append(timeit(fn))
    errs = {}
    for k, fn in runs.items():
        fn()
        torch.cuda.synchronize()
        errs[k] = check()
    print(f"{name:24s} " + " ".join(f"{k}={flops / sorted(v)[1] / 1e9:.0f}({errs[k]:.1e})" for k, v in res.items()),
          flush=True)


for name, M, N, K in [("qkv640", 65536, 1920, 640), ("qkv1280", 16384, 3840, 1280), ("q640", 65536, 640, 640),
                      ("q1280", 16384, 1280, 1280)]:
    a = torch.randn(M, K, device=dev).to(torch.bfloat16)
    w = (torch.randn(N, K, device=dev) / math.sqrt(K)).to(torch.bfloat16)
    b = torch.randn(N, device=dev).to(torch.bfloat16)
    out = torch.empty(M, N, device=dev, dtype=torch.bfloat16)
    ws = core._v7_ws(M, N, K, dev)
    rs = core.layernorm_stats(a, 1e-5)
    cs = w.float().sum(dim=1).contiguous()
    ref = a[:512].float() @ w.float().t() + b.float()
    mu, rstd = rs[:512, 0:1], rs[:512, 1:2]
    ref_ln = rstd * (a[:512].float() @ w.float().t() - mu * cs) + b.float()
    chk = lambda: ((out[:512].float() - ref).norm() / ref.norm()).item()  # noqa: E731
    chk_ln = lambda: ((out[:512].float() - ref_ln).norm() / ref_ln.norm()).item()  # noqa: E731

    def plain(v):
        if v == 7 and ws is not None:
            return lib.cgs_gemm_bf16_v7ws(a.data_ptr(), w.data_ptr(), out.data_ptr(), b.data_ptr(), None, M, N, K, K, K,
                                          N, 0, core.EPI_BIAS, 1.0, ws.data_ptr(), ws.numel(), core._stream())
        return lib.cgs_gemm_bf16_v(a.data_ptr(), w.data_ptr(), out.data_ptr(), b.data_ptr(), None, M, N, K, K, K, N, 0,
                                   core.EPI_BIAS, 1.0, v, core._stream())

    def ln(v):
        return lib.cgs_gemm_bf16_lnfold_v(a.data_ptr(), w.data_ptr(), out.data_ptr(), b.data_ptr(), rs.data_ptr(),
                                          cs.data_ptr(), M, N, K, K, K, N, core.EPI_BIAS,
                                          None if ws is None else ws.data_ptr(), 0 if ws is None else ws.numel(), v,
                                          core._stream())
    ab(name, 2.0 * M * N * K, {"v6": lambda: plain(6), "v7": lambda: plain(7), "v5": lambda: plain(5)}, chk)
    ab("ln:" + name, 2.0 * M * N * K, {"v6": lambda: ln(6), "v7": lambda: ln(7)}, chk_ln)
    del a, w, out, ws

CONVS = [("L1 res 640", 16, 64, 64, 640, 640, 3, 1), ("L1 out-res 1920->640", 16, 64, 64, 1920, 640, 3, 1),
         ("L1 out-res 1280->640", 16, 64, 64, 1280, 640, 3, 1), ("L1 down s2", 16, 64, 64, 640, 640, 3, 2),
         ("L1 res 320->640", 16, 64, 64, 320, 640, 3, 1), ("up conv 640 @128", 16, 128, 128, 640, 640, 3, 1),
         ("L2 res 1280", 16, 32, 32, 1280, 1280, 3, 1)]
for name, N, H, W, Cin, Cout, k, s in CONVS:
    p = k // 2
    x = (torch.rand(N, H, W, Cin, device=dev) * 2 - 1).to(torch.bfloat16)
    w = ((torch.rand(Cout, k, k, Cin, device=dev) * 2 - 1) / math.sqrt(Cin * k * k)).to(torch.bfloat16)
    b = torch.zeros(Cout, device=dev, dtype=torch.bfloat16)
    Ho, Wo = (H + 2 * p - k) // s + 1, (W + 2 * p - k) // s + 1
    out = torch.empty(N, Ho, Wo, Cout, device=dev, dtype=torch.bfloat16)
    ref = torch.nn.functional.conv2d(x[:1].permute(0, 3, 1, 2).float(), w.permute(0, 3, 1, 2).float(), None, s, p)
    ref = ref.permute(0, 2, 3, 1)
    nws = lib.cgs_v7_ws_bytes(N * Ho * Wo, Cout, k * k * Cin)
    ws = torch.empty(max(nws, 1), dtype=torch.uint8, device=dev)

    def cv(v):
        if v == 77:
            return lib.cgs_conv2d_nhwc_v7ws(x.data_ptr(), None, Cin, w.data_ptr(), b.data_ptr(), None, out.data_ptr(),
                                            N, H, W, Cin, Cout, k, k, s, p, Ho, Wo, 0, ws.data_ptr(), nws,
                                            core._stream())
        return lib.cgs_conv2d_nhwc_v(x.data_ptr(), None, Cin, w.data_ptr(), b.data_ptr(), None, out.data_ptr(), N, H, W,
                                     Cin, Cout, k, k, s, p, Ho, Wo, 0, v, core._stream())
    ab(name, 2.0 * N * Ho * Wo * Cout * Cin * k * k, {"v5": lambda: cv(5), "v6": lambda: cv(6), "v7s": lambda: cv(77)},
       lambda: ((out[:1].float() - ref).norm() / ref.norm()).item())
    del x, w, out, ws
