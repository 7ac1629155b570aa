"""SURVEY K06 "GroupNorm into the next conv's prologue", measured: the v6 conv with the input's GroupNorm + SiLU
applied to its A fragments after the LDS read (cgs_conv2d_nhwc_gna_probe: per-element fma + exp2 + rcp + mul on
the fragments each wave reads; padding taps not kept zero, so the time is a LOWER bound for the fused form) vs the
unfused pair it would replace: the GroupNorm apply pass (cgs_groupnorm_apply_stats: (scale, shift) from the
statistics + one read / write of the tensor) + the plain v6 conv. SDXL UNet ResBlock conv shapes at batch 16;
one process, interleaved, median of 5.

python tools/probes/conv_gn_prologue.py  (needs profiles/r06/conv_gn_prologue_experiment.patch applied: the timing-only
kernel is not kept in the library)"""
import os
import statistics
import sys

import torch

sys.path.insert(0, os.getcwd())
from comfy_gen_server_amd.ops import core  # noqa: E402

dev = torch.device("cuda", 0)
lib = core._lib()
s = core._stream()


def _t(f, n=10):
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
for name, N, H, Cin, Cout in [("L0 320", 16, 128, 320, 320), ("L1 640", 16, 64, 640, 640),
                              ("L2 1280", 16, 32, 1280, 1280), ("L1 960->640 (decoder)", 16, 64, 960, 640)]:
    x = torch.randn(N, H, H, Cin, device=dev).to(torch.bfloat16)
    w = (torch.randn(Cout, 3, 3, Cin, device=dev) / (9 * Cin) ** 0.5).to(torch.bfloat16)
    b = torch.randn(Cout, device=dev).to(torch.bfloat16)
    y = torch.empty(N, H, H, Cout, device=dev, dtype=torch.bfloat16)
    xn = torch.empty_like(x)
    gamma = torch.randn(Cin, device=dev).to(torch.bfloat16)
    beta = torch.randn(Cin, device=dev).to(torch.bfloat16)
    mr = torch.stack([torch.randn(N * 32, device=dev), torch.rand(N * 32, device=dev) + 0.5], 1).contiguous()
    ab = torch.empty(N * Cin * 2, device=dev, dtype=torch.float32)
    gna = torch.stack([torch.rand(N, Cin, device=dev) + 0.5, torch.randn(N, Cin, device=dev)], 2).contiguous()

    def apply():
        assert lib.cgs_groupnorm_apply_stats(x.data_ptr(), None, Cin, xn.data_ptr(), gamma.data_ptr(),
                                             beta.data_ptr(), None, mr.data_ptr(), ab.data_ptr(), N, H * H, Cin, 32, 1,
                                             1, s) == 0

    def conv():
        assert lib.cgs_conv2d_nhwc_v(xn.data_ptr(), None, Cin, w.data_ptr(), b.data_ptr(), None, y.data_ptr(), N, H,
                                     H, Cin, Cout, 3, 3, 1, 1, H, H, 0, 6, s) == 0

    def fused():
        assert lib.cgs_conv2d_nhwc_gna_probe(x.data_ptr(), w.data_ptr(), b.data_ptr(), y.data_ptr(), N, H, H, Cin,
                                             Cout, gna.data_ptr(), s) == 0
    ts = {"apply": [], "conv": [], "fused": []}
    for _ in range(5):
        for k, f in (("apply", apply), ("conv", conv), ("fused", fused)):
            ts[k].append(_t(f))
    m = {k: statistics.median(v) for k, v in ts.items()}
    fl = 2.0 * N * H * H * Cin * Cout * 9
    print(f"{name}: apply {m['apply']:.1f} us + v6 conv {m['conv']:.1f} us ({fl / m['conv'] / 1e6:.0f} TF/s) = "
          f"{m['apply'] + m['conv']:.1f} us  vs  fused (lower bound) {m['fused']:.1f} us "
          f"({fl / m['fused'] / 1e6:.0f} TF/s): fused {m['fused'] / (m['apply'] + m['conv']) - 1:+.1%}", flush=True)
