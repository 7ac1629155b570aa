"""Per-shape GEMM table on the SDXL bench shapes: every HIP variant vs hipBLASLt (through ATen).

python -m comfy_gen_server_amd.tools.gemm_table [out.md] [--iters N]

Shapes are the UNet Linear layers of SDXL at 1024x1024 with the CFG-doubled batch of 8 images per
GPU (UNet batch 16): M = 16*64*64 = 65536 tokens at 640 channels, 16*32*32 = 16384 at 1280.
"""
from __future__ import annotations

import math
import sys

import torch

SHAPES = [
    # (name, M, N, K, residual, geglu)
    ("qkv640", 65536, 1920, 640, False, False),
    ("out640+res", 65536, 640, 640, True, False),
    ("q640", 65536, 640, 640, False, False),
    ("geglu640", 65536, 5120, 640, False, True),
    ("ffout640+res", 65536, 640, 2560, True, False),
    ("qkv1280", 16384, 3840, 1280, False, False),
    ("out1280+res", 16384, 1280, 1280, True, False),
    ("q1280", 16384, 1280, 1280, False, False),
    ("geglu1280", 16384, 10240, 1280, False, True),
    ("ffout1280+res", 16384, 1280, 5120, True, False),
    ("kv_ctx1280", 1232, 2560, 2048, False, False),
]

VARIANTS = {"v5": 5, "v6": 6, "v7": 7, "v7s": 8, "v4": 4, "w6": 16, "w6n160": 17, "v6w4": 20, "auto": -1}
# v7s: v7 + split-K tail; w6: one wave per SIMD, 256 x 256 (w6n160: 256 x 160); v6w4: 128 x 80, 4 waves


def _time(fn, iters):
    for _ in range(2):
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
    import torch.nn.functional as F
    from comfy_gen_server_amd import _native
    from comfy_gen_server_amd.ops import core
    iters = 20
    if "--iters" in argv:
        i = argv.index("--iters")
        iters = int(argv[i + 1])
        argv = argv[:i] + argv[i + 2:]
    lib = _native.load_kernels()
    assert lib is not None, _native.kernels_error()
    dev = torch.device("cuda", 0)
    rows = ["| shape | M | N | K | " + " | ".join(f"{v} TF/s" for v in VARIANTS) + " | hipBLASLt TF/s | best |",
            "|---|---:|---:|---:|" + "---:|" * (len(VARIANTS) + 2)]
    for name, M, N, K, res, geglu in SHAPES:
        a = torch.randn(M, K, device=dev).to(torch.bfloat16)
        w = (torch.randn(N, K, device=dev) / math.sqrt(K)).to(torch.bfloat16)
        b = torch.randn(N, device=dev).to(torch.bfloat16)
        r = torch.randn(M, N // (2 if geglu else 1), device=dev).to(torch.bfloat16) if res else None
        flops = 2.0 * M * N * K
        epi = core.EPI_BIAS | (core.EPI_RESIDUAL if res else 0) | (core.EPI_GEGLU if geglu else 0)
        nout = N // 2 if geglu else N
        out = torch.empty(M, nout, device=dev, dtype=torch.bfloat16)
        ref = None
        res_tf = {}
        for vname, v in VARIANTS.items():
            nws = lib.cgs_v7_ws_bytes(M, N, K)
            ws = torch.empty(max(nws, 1), dtype=torch.uint8, device=dev)

            def run(v=v):
                if v == 8:
                    return lib.cgs_gemm_bf16_v7ws(a.data_ptr(), w.data_ptr(), out.data_ptr(), b.data_ptr(),
                                                  None if r is None else r.data_ptr(), M, N, K, K, K, nout,
                                                  nout if r is not None else 0, epi, 1.0, ws.data_ptr(), nws,
                                                  core._stream())
                return lib.cgs_gemm_bf16_v(a.data_ptr(), w.data_ptr(), out.data_ptr(), b.data_ptr(),
                                           None if r is None else r.data_ptr(), M, N, K, K, K, nout,
                                           nout if r is not None else 0, epi, 1.0, v, core._stream())
            try:
                if run() != 0:
                    raise RuntimeError("launch failed")
                torch.cuda.synchronize()
                if ref is None:
                    wf = core.geglu_deinterleave(w).float() if geglu else w.float()
                    bf = core.geglu_deinterleave(b).float() if geglu else b.float()
                    h = a[:4096].float() @ wf.t() + bf
                    if geglu:
                        x1, g = h.chunk(2, dim=-1)
                        h = x1 * F.gelu(g)
                    ref = h + (r[:4096].float() if r is not None else 0)
                err = ((out[:4096].float() - ref).norm() / ref.norm()).item()
                ms = _time(run, iters)
                res_tf[vname] = flops / ms / 1e9 if err < 2e-2 else -1.0
            except Exception:
                res_tf[vname] = float("nan")
        if geglu:
            lib_fn = lambda: F.linear(a, w, b)  # noqa: E731  (no fused gate: lower bound for the library)
        else:
            lib_fn = (lambda: F.linear(a, w, b).add_(r)) if r is not None else (lambda: F.linear(a, w, b))
        ms = _time(lib_fn, iters)
        res_tf["lib"] = flops / ms / 1e9
        best = max(res_tf, key=lambda k: res_tf[k] if res_tf[k] == res_tf[k] else -2)
        rows.append(f"| {name} | {M} | {N} | {K} | " + " | ".join(
            ("bad" if res_tf[v] == -1.0 else f"{res_tf[v]:.0f}") for v in VARIANTS) +
            f" | {res_tf['lib']:.0f} | {best} |")
        print(rows[-1], flush=True)
        del a, w, b, r, out
    text = "\n".join(rows)
    if argv:
        with open(argv[0], "w") as f:
            f.write(text + "\n")
    print(text)


if __name__ == "__main__":
    main(sys.argv[1:])
