"""What the GroupNorm-statistics epilogue costs the v6 conv (cgs_conv2d_nhwc_gns vs cgs_conv2d_nhwc_v variant 6,
same shape, bias, no residual) on the SDXL UNet conv1 shapes at batch 16, in one process, interleaved; plus
the standalone statistics pass it replaces (cgs_groupnorm_band_stats over the conv output).

python tools/probes/conv_gns_cost.py
"""
import statistics
import sys

import torch

sys.path.insert(0, __file__.rsplit("/tools/", 1)[0])

from comfy_gen_server_amd import _native  # noqa: E402
from comfy_gen_server_amd.ops import core  # noqa: E402

SHAPES = [("L0 res 320", 16, 128, 320, 320), ("L0 out 960->320", 16, 128, 960, 320),
          ("L1 res 640", 16, 64, 640, 640), ("L1 out 1920->640", 16, 64, 1920, 640),
          ("L2 res 1280", 16, 32, 1280, 1280), ("L2 out 2560->1280", 16, 32, 2560, 1280)]


def _t(f, n=10):
    for _ in range(2):
        f()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(n):
        f()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / n * 1e3


def main():
    lib = _native.load_kernels()
    assert lib is not None and _native.has_kernel("cgs_conv2d_nhwc_gns"), _native.kernels_error()
    dev = torch.device("cuda", 0)
    st = core._stream()
    torch.manual_seed(0)
    for name, N, HW, Cin, Cout in SHAPES:
        x = torch.randn(N, HW, HW, Cin, device=dev).to(torch.bfloat16)
        w = (0.02 * torch.randn(Cout, 3, 3, Cin, device=dev)).to(torch.bfloat16)
        b = torch.randn(Cout, device=dev).to(torch.bfloat16)
        out = torch.empty(N, HW, HW, Cout, device=dev, dtype=torch.bfloat16)
        part = torch.empty(N * (HW * HW // 64) * Cout * 2, device=dev, dtype=torch.float32)
        wsb = int(lib.cgs_groupnorm_workspace(N, HW * HW, Cout))
        ws = torch.empty((wsb + 3) // 4, device=dev, dtype=torch.float32)
        stats = torch.empty(N * 32 * 2, device=dev, dtype=torch.float32)
        args = (x.data_ptr(), None, Cin, w.data_ptr(), b.data_ptr(), None, out.data_ptr(), N, HW, HW, Cin, Cout, 3, 3,
                1, 1, HW, HW, 1)

        def plain():
            assert lib.cgs_conv2d_nhwc_v(*args, 6, st) == 0

        def gns():
            assert lib.cgs_conv2d_nhwc_gns(*args, part.data_ptr(), st) == 0

        def stats_pass():
            assert lib.cgs_groupnorm_band_stats(out.data_ptr(), None, Cout, None, ws.data_ptr(), stats.data_ptr(), N,
                                                HW * HW, Cout, 32, 1, st) == 0
        ts = {"plain": [], "gns": [], "stats": []}
        for _ in range(5):
            ts["plain"].append(_t(plain))
            ts["gns"].append(_t(gns))
            ts["stats"].append(_t(stats_pass))
        us = {k: statistics.median(v) for k, v in ts.items()}
        fl = 2.0 * N * HW * HW * Cin * Cout * 9
        print(f"{name}: v6 {us['plain']:.1f} us ({fl / us['plain'] / 1e6:.0f} TF/s)  v6+GNS {us['gns']:.1f} us "
              f"({us['gns'] / us['plain'] - 1:+.1%})  stats pass {us['stats']:.1f} us  "
              f"-> GNS saves {us['plain'] + us['stats'] - us['gns']:.1f} us", flush=True)


if __name__ == "__main__":
    main()
