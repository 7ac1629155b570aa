"""Per-shape conv table on the SDXL bench shapes (UNet batch 16 at 1024^2, VAE decode batch 8):
every HIP conv variant vs MIOpen (F.conv2d, channels_last) in TF/s.

python -m comfy_gen_server_amd.tools.conv_table [out.md] [--vae] [--miopen] [--gemm]

``--gemm`` adds the same-sized plain GEMM (M = N*Ho*Wo, N = Cout, K = k*k*Cin; im2col already done) on
hipBLASLt (torch.mm) and on our GEMM (ops.linear): the rate an implicit-GEMM conv is chasing.
"""
from __future__ import annotations

import math
import sys

import torch
import torch.nn.functional as F

UNET = [  # (name, N, H, W, Cin, Cout, k, stride)
    ("L0 res 320", 16, 128, 128, 320, 320, 3, 1),
    ("L0 out-res 960->320", 16, 128, 128, 960, 320, 3, 1),
    ("L0 out-res 640->320", 16, 128, 128, 640, 320, 3, 1),
    ("L0 down s2", 16, 128, 128, 320, 320, 3, 2),
    ("L1 res 320->640", 16, 64, 64, 320, 640, 3, 1),
    ("L1 res 640", 16, 64, 64, 640, 640, 3, 1),
    ("L1 out-res 1920->640", 16, 64, 64, 1920, 640, 3, 1),
    ("L1 out-res 1280->640", 16, 64, 64, 1280, 640, 3, 1),
    ("L1 out-res 960->640", 16, 64, 64, 960, 640, 3, 1),
    ("L1 down s2", 16, 64, 64, 640, 640, 3, 2),
    ("L2 res 640->1280", 16, 32, 32, 640, 1280, 3, 1),
    ("L2 res 1280", 16, 32, 32, 1280, 1280, 3, 1),
    ("L2 out-res 2560->1280", 16, 32, 32, 2560, 1280, 3, 1),
    ("L2 out-res 1920->1280", 16, 32, 32, 1920, 1280, 3, 1),
    ("up conv 1280 @64", 16, 64, 64, 1280, 1280, 3, 1),
    ("up conv 640 @128", 16, 128, 128, 640, 640, 3, 1),
    ("skip 1x1 960->320", 16, 128, 128, 960, 320, 1, 1),
    ("2x-up conv 1280 32->64", 16, 32, 32, 1280, 1280, 3, 1),     # "2x": input read through nearest-2x
    ("2x-up conv 640 64->128", 16, 64, 64, 640, 640, 3, 1),
]
VAE = [
    ("vae 512 @128", 8, 128, 128, 512, 512, 3, 1),
    ("vae 512 @256", 8, 256, 256, 512, 512, 3, 1),
    ("vae 512 @512", 8, 512, 512, 512, 512, 3, 1),
    ("vae 512->256 @512", 8, 512, 512, 512, 256, 3, 1),
    ("vae 256 @512", 8, 512, 512, 256, 256, 3, 1),
    ("vae 256 @1024", 8, 1024, 1024, 256, 256, 3, 1),
    ("vae 256->128 @1024", 8, 1024, 1024, 256, 128, 3, 1),
    ("vae 128 @1024", 8, 1024, 1024, 128, 128, 3, 1),
    ("vae 2x-up 512 128->256", 8, 128, 128, 512, 512, 3, 1),
    ("vae 2x-up 256 512->1024", 8, 512, 512, 256, 256, 3, 1),
]
# v7s: v7 + split-K tail; v6k: v6 with the older per-lane-address gather (ConvGatherK) instead of ConvGatherKD
VARIANTS = {"v2": 2, "v5": 5, "v6": 6, "v6k": 16, "v6n128": 18, "v6w4": 21, "v7": 7, "v7s": 8}


def _time(fn, iters):
    fn()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(iters):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / iters


def main(argv):
    from comfy_gen_server_amd import _native
    from comfy_gen_server_amd.ops import core
    lib = _native.load_kernels()
    dev = torch.device("cuda", 0)
    shapes = UNET + (VAE if "--vae" in argv else [])
    gemm = "--gemm" in argv
    argv = [a for a in argv if a not in ("--vae", "--miopen", "--gemm")]
    rows = ["| conv | N | HxW | Cin | Cout | k/s | " + " | ".join(f"{v} TF/s" for v in VARIANTS) + " | MIOpen TF/s |"
            + (" GEMM hipBLASLt | GEMM ours | GEMM v6 |" if gemm else ""),
            "|---|---:|---|---:|---:|---|" + "---:|" * (len(VARIANTS) + 1 + 3 * gemm)]
    for name, N, H, W, Cin, Cout, k, s in shapes:
        p = k // 2
        up = "2x" in name
        fl = 16 if up else 0
        x = (torch.rand(N, Cin, H, W, device=dev) * 2 - 1).to(torch.bfloat16).contiguous(memory_format=torch.channels_last)
        w = ((torch.rand(Cout, Cin, k, k, device=dev) * 2 - 1) / math.sqrt(Cin * k * k)).to(torch.bfloat16)
        wn = w.permute(0, 2, 3, 1).contiguous()
        b = torch.zeros(Cout, device=dev, dtype=torch.bfloat16)
        Hl, Wl = (2 * H, 2 * W) if up else (H, W)
        Ho, Wo = (Hl + 2 * p - k) // s + 1, (Wl + 2 * p - k) // s + 1
        out = torch.empty(N, Cout, Ho, Wo, device=dev, dtype=torch.bfloat16, memory_format=torch.channels_last)
        flops = 2.0 * N * Ho * Wo * Cout * Cin * k * k
        it = max(2, int(3e11 / flops))
        x1 = x[:1].float()
        ref = F.conv2d(F.interpolate(x1, scale_factor=2, mode="nearest") if up else x1, w.float(), b.float(), s, p)
        res = {}
        nws = lib.cgs_v7_ws_bytes(N * Ho * Wo, Cout, k * k * Cin)
        ws = torch.empty(max(nws, 1), dtype=torch.uint8, device=dev)
        for vn, v in VARIANTS.items():
            def run(v=v):
                if v == 16:
                    lib.cgs_conv_v6_set_loader(1)
                    try:
                        return lib.cgs_conv2d_nhwc_v(x.data_ptr(), None, Cin, wn.data_ptr(), b.data_ptr(), None,
                                                     out.data_ptr(), N, H, W, Cin, Cout, k, k, s, p, Ho, Wo, fl, 6,
                                                     core._stream())
                    finally:
                        lib.cgs_conv_v6_set_loader(-1)
                if v == 8:
                    return lib.cgs_conv2d_nhwc_v7ws(x.data_ptr(), None, Cin, wn.data_ptr(), b.data_ptr(), None,
                                                    out.data_ptr(), N, H, W, Cin, Cout, k, k, s, p, Ho, Wo, fl,
                                                    ws.data_ptr(), nws, core._stream())
                return lib.cgs_conv2d_nhwc_v(x.data_ptr(), None, Cin, wn.data_ptr(), b.data_ptr(), None,
                                             out.data_ptr(), N, H, W, Cin, Cout, k, k, s, p, Ho, Wo, fl, v,
                                             core._stream())
            try:
                if run() != 0:
                    res[vn] = float("nan")
                    continue
                torch.cuda.synchronize()
                err = ((out[:1].float() - ref).norm() / ref.norm()).item()
                res[vn] = flops / _time(run, it) / 1e9 if err < 2e-2 else -1.0
            except Exception:
                res[vn] = float("nan")
        if "--miopen" in sys.argv:
            ms = _time(lambda: F.conv2d(F.interpolate(x, scale_factor=2, mode="nearest") if up else x, w, b, s, p),
                       it)
            res["miopen"] = flops / ms / 1e9
        else:
            res["miopen"] = float("nan")
        extra = ""
        if gemm and not up:
            del ws
            ws = None
            A = torch.empty(N * Ho * Wo, k * k * Cin, device=dev, dtype=torch.bfloat16).uniform_(-1, 1)
            Wt = w.reshape(Cout, -1).contiguous()
            t_lib = _time(lambda: torch.mm(A, Wt.t()), it)
            t_our = _time(lambda: core.linear(A, Wt, b), it)
            Cg = torch.empty(A.shape[0], Cout, device=dev, dtype=torch.bfloat16)
            Kg = A.shape[1]

            def v6():   # the conv's v6 main loop on a row-major A (the im2col-free loader's cost is the difference)
                return lib.cgs_gemm_bf16_v(A.data_ptr(), Wt.data_ptr(), Cg.data_ptr(), b.data_ptr(), None, A.shape[0],
                                           Cout, Kg, Kg, Kg, Cout, 0, 1, 1.0, 6, core._stream())
            t_v6 = _time(v6, it) if Cout % 160 == 0 and v6() == 0 else float("nan")
            extra = f" {flops / t_lib / 1e9:.0f} | {flops / t_our / 1e9:.0f} | {flops / t_v6 / 1e9:.0f} |"
            del Cg
            del A
        elif gemm:
            extra = " | | |"
        rows.append(f"| {name} | {N} | {H}x{W} | {Cin} | {Cout} | {k}/{s} | " +
                    " | ".join("bad" if res[v] == -1.0 else f"{res[v]:.0f}" for v in VARIANTS) +
                    f" | {res['miopen']:.0f} |" + extra)
        print(rows[-1], flush=True)
        del x, w, wn, out, ws
    text = "\n".join(rows)
    if argv:
        open(argv[0], "w").write(text + "\n")
    print(text)


if __name__ == "__main__":
    main(sys.argv[1:])
