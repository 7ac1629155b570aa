"""The 256 x 128 v6 conv tile (variant 18; the prefetch arm needs the cgs_conv_n128_set_pfe toggle this was measured
with -- removed after it lost) vs the 256 x 160
v6 tile (variant 6) and the 256 x 256 v5 tile (variant 5) on the SDXL VAE decoder shapes (batch 8), with and
without the ResnetBlock residual; one process, interleaved, median of 5; outputs checked against the v6 result.

python tools/probes/conv_n128_ab.py"""
import os
import statistics
import sys

import torch

sys.path.insert(0, os.getcwd())
from comfy_gen_server_amd.ops import core  # noqa: E402

dev = torch.device("cuda", 0)
lib = core._lib()
SHAPES = [(8, 1024, 128, 128, True), (8, 1024, 128, 128, False), (8, 1024, 256, 128, False),
          (8, 512, 256, 256, True), (8, 512, 512, 256, False), (8, 256, 512, 512, True), (8, 128, 512, 512, True)]


def _t(f, n=5):
    f()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(n):
        f()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / n


for N, H, Cin, Cout, res in SHAPES:
    x = (torch.rand(N, H, H, Cin, device=dev) * 2 - 1).to(torch.bfloat16)
    w = ((torch.rand(Cout, 3, 3, Cin, device=dev) * 2 - 1) / (9 * Cin) ** 0.5).to(torch.bfloat16)
    b = torch.randn(Cout, device=dev).to(torch.bfloat16)
    r = torch.randn(N, H, H, Cout, device=dev).to(torch.bfloat16) if res else None
    outs = {}

    def run(v, pfe=1):
        lib.cgs_conv_n128_set_pfe(pfe)
        o = outs.setdefault((v, pfe), torch.empty(N, H, H, Cout, device=dev, dtype=torch.bfloat16))
        assert lib.cgs_conv2d_nhwc_v(x.data_ptr(), None, Cin, w.data_ptr(), b.data_ptr(), core._ptr(r), o.data_ptr(),
                                     N, H, H, Cin, Cout, 3, 3, 1, 1, H, H, 0, v, core._stream()) == 0
    cfgs = [("v6", 6, 1), ("v5", 5, 1), ("n128", 18, 0), ("n128+pf", 18, 1)]
    ts = {c[0]: [] for c in cfgs}
    for _ in range(5):
        for name, v, pfe in cfgs:
            ts[name].append(_t(lambda: run(v, pfe)))
    lib.cgs_conv_n128_set_pfe(1)
    ref = outs[(6, 1)].float()
    fl = 2.0 * N * H * H * Cin * Cout * 9
    line = "  ".join(f"{n} {statistics.median(t):.3f} ms ({fl / statistics.median(t) / 1e9:.0f} TF/s)"
                     for n, t in ts.items())
    err = max(((outs[(v, p)].float() - ref).norm() / ref.norm()).item() for _, v, p in cfgs)
    print(f"N={N} {H}x{H} {Cin}->{Cout} res={res}: {line}  max rel diff vs v6 {err:.2e}", flush=True)
    assert err < 1e-2
    del x, w, r, outs
    torch.cuda.empty_cache()
