"""Narrow-output conv (Cout <= 16): the LDS-staged halo form vs the direct-load form (cgs_conv_smalln_set_lds), on
the SDXL VAE decoder's conv_out (8 x 1024^2, 128 -> 3) and the UNet's conv_out (16 x 128^2, 320 -> 4); one process,
interleaved, median of 5; the two outputs must be bitwise equal (same MFMA order per tap and chunk)."""
import os
import statistics
import sys

import torch

sys.path.insert(0, os.getcwd())
from comfy_gen_server_amd.ops import core  # noqa: E402

dev = torch.device("cuda", 0)
lib = core._lib()
for N, H, W, Cin, Cout, res in [(8, 1024, 1024, 128, 3, False), (1, 1024, 1024, 128, 3, False),
                                (16, 128, 128, 320, 4, False), (2, 130, 70, 64, 16, True)]:
    x = torch.randn(N, H, W, Cin, device=dev).to(torch.bfloat16)
    w = (torch.randn(Cout, 3, 3, Cin, device=dev) / (9 * Cin) ** 0.5).to(torch.bfloat16)
    b = torch.randn(Cout, device=dev).to(torch.bfloat16)
    r = torch.randn(N, H, W, Cout, device=dev).to(torch.bfloat16) if res else None
    outs = {m: torch.empty(N, H, W, Cout, device=dev, dtype=torch.bfloat16) for m in (0, 1)}

    def run(m):
        lib.cgs_conv_smalln_set_lds(m)
        assert lib.cgs_conv2d_nhwc_v(x.data_ptr(), None, Cin, w.data_ptr(), b.data_ptr(), core._ptr(r),
                                     outs[m].data_ptr(), N, H, W, Cin, Cout, 3, 3, 1, 1, H, W, 1 | (2 if res else 0),
                                     -2, core._stream()) == 0
    ts = {0: [], 1: []}
    for _ in range(5):
        for m in (0, 1):
            run(m)
            torch.cuda.synchronize()
            s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            s.record()
            for _ in range(5):
                run(m)
            e.record()
            torch.cuda.synchronize()
            ts[m].append(s.elapsed_time(e) / 5)
    lib.cgs_conv_smalln_set_lds(1)
    gb = N * H * W * Cin * 2 / 1e9
    line = "  ".join(f"{'lds' if m else 'direct'} {statistics.median(t):.3f} ms ({gb / statistics.median(t):.2f} TB/s of input)"
                     for m, t in ts.items())
    print(f"N={N} {H}x{W} {Cin}->{Cout} res={res}: {line}  bitwise-equal={torch.equal(outs[0], outs[1])}", flush=True)
