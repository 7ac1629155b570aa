"""Measured A/B of GroupNorm statistics in the producing conv's epilogue (K06 second half):
  A: v6 conv -> GroupNorm (gn_partial over the conv output + finalize + apply, +SiLU)
  B: v6 conv with the statistics epilogue (cgs_conv2d_nhwc_gns) -> finalize + apply
Prints per-part and end-to-end times (median of 3 interleaved rounds) and max |y_A - y_B|."""
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
    return s.elapsed_time(e) / iters * 1e3


SHAPES = [("L0 res 320", 16, 128, 128, 320, 320), ("L0 out-res 960->320", 16, 128, 128, 960, 320),
          ("L1 res 640 (v6)", 16, 64, 64, 640, 640), ("L2 res 1280 (v6)", 16, 32, 32, 1280, 1280)]
for name, N, H, W, Cin, Cout in SHAPES:
    x = (torch.rand(N, H, W, Cin, device=dev) * 2 - 1).to(torch.bfloat16)
    w = ((torch.rand(Cout, 3, 3, Cin, device=dev) * 2 - 1) / math.sqrt(Cin * 9)).to(torch.bfloat16)
    b = (torch.randn(Cout, device=dev) * 0.5).to(torch.bfloat16)
    gamma = (1 + 0.1 * torch.randn(Cout, device=dev)).to(torch.bfloat16)
    beta = (0.1 * torch.randn(Cout, device=dev)).to(torch.bfloat16)
    out = torch.empty(N, H, W, Cout, device=dev, dtype=torch.bfloat16)
    ya = torch.empty_like(out)
    yb = torch.empty_like(out)
    HW = H * W
    ws = torch.empty(int(lib.cgs_groupnorm_workspace(N, HW, Cout)), dtype=torch.uint8, device=dev)
    gnp = torch.empty(N * (HW // 64) * Cout * 2, dtype=torch.float32, device=dev)
    ab = torch.empty(N * Cout * 2, dtype=torch.float32, device=dev)
    st = core._stream()

    def conv_a():
        assert lib.cgs_conv2d_nhwc_v(x.data_ptr(), None, Cin, w.data_ptr(), b.data_ptr(), None, out.data_ptr(), N, H, W,
                                     Cin, Cout, 3, 3, 1, 1, H, W, 0, 6, st) == 0

    def conv_b():
        assert lib.cgs_conv2d_nhwc_gns(x.data_ptr(), None, Cin, w.data_ptr(), b.data_ptr(), None, out.data_ptr(), N, H,
                                       W, Cin, Cout, 3, 3, 1, 1, H, W, 0, gnp.data_ptr(), st) == 0

    def gn_a():
        assert lib.cgs_groupnorm_nhwc_ws(out.data_ptr(), ya.data_ptr(), gamma.data_ptr(), beta.data_ptr(), None,
                                         ws.data_ptr(), N, HW, Cout, 32, 1e-5, 1, 1, st) == 0

    def gn_b():
        assert lib.cgs_groupnorm_nhwc_part(out.data_ptr(), yb.data_ptr(), gamma.data_ptr(), beta.data_ptr(), None,
                                           gnp.data_ptr(), ab.data_ptr(), N, HW, Cout, 32, 64, 1e-5, 1, 1, st) == 0

    runs = {"convA": conv_a, "convB+stats": conv_b, "gnA(partial+fin+apply)": gn_a, "gnB(fin+apply)": gn_b,
            "A=conv+gn": lambda: (conv_a(), gn_a()), "B=convstats+gn": lambda: (conv_b(), gn_b())}
    res = {k: [] for k in runs}
    for _ in range(3):
        for k, fn in runs.items():
            res[k].append(timeit(fn))
    conv_a(); gn_a(); conv_b(); gn_b()
    torch.cuda.synchronize()
    ref = torch.nn.functional.silu(torch.nn.functional.group_norm(out.permute(0, 3, 1, 2).float(), 32,
                                                                  gamma.float(), beta.float(), 1e-5)).permute(0, 2, 3, 1)
    d_ab = (ya.float() - yb.float()).abs().max().item()
    d_ref = (yb.float() - ref).abs().max().item()
    print(f"{name:22s} " + " ".join(f"{k}={sorted(v)[1]:.1f}us" for k, v in res.items()) +
          f" | max|yA-yB|={d_ab:.3g} max|yB-fp32|={d_ref:.3g}", flush=True)
    del x, w, out, ya, yb, ws, gnp
