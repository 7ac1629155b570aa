"""In-process interleaved A/B of the GEMM kernels on the SDXL shapes (the one-wave-per-SIMD w6 -- persistent,
non-persistent, 256x160 -- vs the 8-wave v6 / v7 kernels vs hipBLASLt through ATen), with an fp32 numerics
check of every HIP variant.

python -m comfy_gen_server_amd.tools.gemm_ab [out.md] [--rounds R] [--iters N] [--shapes a,b,...] [--v6modes 1,65]
    [--cmp path/to/other/libcgs_kernels.so]

``--v6modes``: extra columns "v6m<m>" = v6 under cgs_v6_set_mode(m) (pq::run DS bits; 64 / 128 = A / B DMAs
through buffer descriptors), interleaved with the others in the same rounds.

Rows are (name, M, N, K, epilogue): epilogue "" plain + bias, "res" + residual, "geglu" (16-row
interleaved a/g weights, N/2 outputs), "ln" (LayerNorm folded in, W' = W * gamma), "ln:geglu".
hipBLASLt runs the un-fused GEMM (bias fused, no residual / gate / LayerNorm: a lower bound of what
the fused op would cost there). TF/s = 2 M N K / time, median over the rounds.
"""
from __future__ import annotations

import math
import statistics
import sys

import torch

SHAPES = [
    ("qkv640", 65536, 1920, 640, "ln"),
    ("out640+res", 65536, 640, 640, "res"),
    ("q640", 65536, 640, 640, "ln"),
    ("geglu640", 65536, 5120, 640, "ln:geglu"),
    ("ffout640+res", 65536, 640, 2560, "res"),
    ("qkv1280", 16384, 3840, 1280, "ln"),
    ("out1280+res", 16384, 1280, 1280, "res"),
    ("q1280", 16384, 1280, 1280, "ln"),
    ("geglu1280", 16384, 10240, 1280, "ln:geglu"),
    ("ffout1280+res", 16384, 1280, 5120, "res"),
    ("kv_ctx1280", 1232, 2560, 2048, ""),
    ("sq8192", 8192, 8192, 8192, ""),
    ("geglu1280-noln", 16384, 10240, 1280, "geglu"),
    ("qkv1280-noln", 16384, 3840, 1280, ""),
]

EPI_BIAS, EPI_RES, EPI_GEGLU, EPI_LN = 1, 2, 4, 8


def _bench(fn, iters):
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    fn()
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
    rounds, iters, only = 3, 10, None
    v6modes = []
    out_md = None
    cmp_path = None
    i = 0
    while i < len(argv):
        if argv[i] == "--rounds":
            rounds = int(argv[i + 1]); i += 2
        elif argv[i] == "--iters":
            iters = int(argv[i + 1]); i += 2
        elif argv[i] == "--shapes":
            only = set(argv[i + 1].split(",")); i += 2
        elif argv[i] == "--cmp":     # another build of the library: its v6 / v7 as columns v6b / v7b
            cmp_path = argv[i + 1]; i += 2
        elif argv[i] == "--v6modes":
            v6modes = [int(v) for v in argv[i + 1].split(",")]; i += 2
        else:
            out_md = argv[i]; i += 1
    lib = _native.load_kernels()
    assert lib is not None, _native.kernels_error()
    lib2 = None
    if cmp_path:
        import ctypes
        lib2 = ctypes.CDLL(cmp_path, mode=ctypes.RTLD_LOCAL)
        _native._declare(lib2)
    dev = torch.device("cuda", 0)
    stream = core._stream()
    rows = ["| shape | M | N | K | epi | w6 TF/s | w6 non-persistent | w6 256x160 | v6 TF/s | v7 TF/s | hipBLASLt TF/s "
            "| best w6 / best other | w6 max rel err |",
            "|---|---:|---:|---:|---|---:|---:|---:|---:|---:|---:|---:|---:|"]
    torch.manual_seed(0)
    for name, M, N, K, epi in SHAPES:
        if only and name not in only:
            continue
        geglu, ln, res = "geglu" in epi, epi.startswith("ln"), epi == "res"
        a = torch.randn(M, K, device=dev).to(torch.bfloat16)
        w = (torch.randn(N, K, device=dev) / math.sqrt(K)).to(torch.bfloat16)
        b = (torch.randn(N, device=dev) * 0.5).to(torch.bfloat16)
        nout = N // 2 if geglu else N
        r = torch.randn(M, nout, device=dev).to(torch.bfloat16) if res else None
        flags = EPI_BIAS | (EPI_RES if res else 0) | (EPI_GEGLU if geglu else 0)
        # fp32 reference (GEGLU on the de-interleaved a / g halves, LayerNorm with gamma / beta)
        if ln:
            gamma = (1.0 + 0.1 * torch.randn(K, device=dev)).to(torch.bfloat16)
            beta = (0.1 * torch.randn(K, device=dev)).to(torch.bfloat16)
            xf = F.layer_norm(a.float(), (K,), gamma.float(), beta.float(), 1e-5)
            w_run, cs, b_run = core.lnfold_weights(w, b, gamma, beta)
            rs = torch.empty(M, 2, device=dev, dtype=torch.float32)
            assert lib.cgs_layernorm_stats(a.data_ptr(), rs.data_ptr(), M, K, 1e-5, 1, stream) == 0
        else:
            xf = a.float()
            w_run, cs, b_run, rs = w, None, b, None
        if geglu:
            w_run = core.geglu_interleave(w_run)
            b_run = core.geglu_interleave(b_run[:, None])[:, 0].contiguous()
        h = xf @ w.float().t() + b.float()
        if geglu:
            ref = h[:, :nout] * F.gelu(h[:, nout:])
        else:
            ref = h + (r.float() if res else 0.0)
        del h, xf
        out = torch.empty(M, nout, device=dev, dtype=torch.bfloat16)
        rp = None if r is None else r.data_ptr()
        ldr = nout if res else 0
        csp = None if cs is None else cs.data_ptr()
        rsp = None if rs is None else rs.data_ptr()

        def var(v, lib=lib):
            def f():
                if ln:
                    e = lib.cgs_gemm_bf16_lnfold_v(a.data_ptr(), w_run.data_ptr(), out.data_ptr(), b_run.data_ptr(),
                                                   rsp, csp, M, N, K, K, K, nout, flags, None, 0, v, stream)
                else:
                    e = lib.cgs_gemm_bf16_v(a.data_ptr(), w_run.data_ptr(), out.data_ptr(), b_run.data_ptr(), rp, M,
                                            N, K, K, K, nout, ldr, flags, 1.0, v, stream)
                return e
            return f
        cands = {}
        if _native.has_kernel("cgs_gemm_bf16_w6") and lib.cgs_gemm_w6_ok(M, N, K, K, K, nout, ldr,
                                                                          flags | (EPI_LN if ln else 0), 256):
            cands["w6"] = lambda: lib.cgs_gemm_bf16_w6(a.data_ptr(), w_run.data_ptr(), out.data_ptr(), b_run.data_ptr(),
                                                       rp, rsp, csp, M, N, K, K, K, nout, ldr,
                                                       flags | (EPI_LN if ln else 0), 1.0, 0, 4, 0, 256, stream)
            cands["w6np"] = lambda: lib.cgs_gemm_bf16_w6(a.data_ptr(), w_run.data_ptr(), out.data_ptr(),
                                                         b_run.data_ptr(), rp, rsp, csp, M, N, K, K, K, nout, ldr,
                                                         flags | (EPI_LN if ln else 0), 1.0, 0, 4, 1 << 30, 256, stream)
        if (_native.has_kernel("cgs_gemm_bf16_w6") and N % 160 == 0 and
                lib.cgs_gemm_w6_ok(M, N, K, K, K, nout, ldr, flags | (EPI_LN if ln else 0), 160)):
            cands["w6n160"] = lambda: lib.cgs_gemm_bf16_w6(a.data_ptr(), w_run.data_ptr(), out.data_ptr(),
                                                           b_run.data_ptr(), rp, rsp, csp, M, N, K, K, K, nout, ldr,
                                                           flags | (EPI_LN if ln else 0), 1.0, 0, 4, 0, 160, stream)
        errs = {}
        for vn, v in (("v6", 6), ("v7", 7)):
            f = var(v)
            if f() == 0:
                cands[vn] = f
        if lib2 is not None:
            for vn, v in (("v6b", 6), ("v7b", 7)):
                f = var(v, lib2)
                if f() == 0:
                    cands[vn] = f
        for m in v6modes:
            def fm(m=m, f6=var(6)):
                lib.cgs_v6_set_mode(m)
                try:
                    return f6()
                finally:
                    lib.cgs_v6_set_mode(-1)
            if fm() == 0:
                cands[f"v6m{m}"] = fm
        cands["lib"] = lambda: F.linear(a, w, b)
        for vn, f in cands.items():
            if vn == "lib":
                continue
            out.zero_()
            assert f() in (0, None), vn
            torch.cuda.synchronize()
            d = (out.float() - ref).abs().max().item()
            errs[vn] = d / max(ref.abs().max().item(), 1e-6)
        times = {vn: [] for vn in cands}
        for _ in range(rounds):
            for vn, f in cands.items():
                times[vn].append(_bench(f, iters))
        flops = 2.0 * M * N * K
        tf = {vn: flops / statistics.median(t) / 1e9 for vn, t in times.items()}
        other = max(v for k, v in tf.items() if not k.startswith(("w4", "w5", "w6")))
        cell = lambda k: f"{tf[k]:.0f}" if k in tf else "-"  # noqa: E731
        bw6 = max(tf.get("w6", 0.0), tf.get("w6n160", 0.0))
        line = (f"| {name} | {M} | {N} | {K} | {epi or 'bias'} | {cell('w6')} | {cell('w6np')} | {cell('w6n160')} | "
                f"{cell('v6')} | {cell('v7')} | {cell('lib')} | {bw6 / other:.3f} | "
                f"{max(errs.get('w6', 0.0), errs.get('w6n160', 0.0)):.2e} |")
        rows.append(line)
        print(line, " errs:", {k: f"{v:.1e}" for k, v in errs.items()}, " TF/s:", {k: round(v) for k, v in tf.items()},
              flush=True)
        del a, w, out, ref
        torch.cuda.empty_cache()
    txt = "\n".join(rows)
    print(txt)
    if out_md:
        with open(out_md, "w") as fh:
            fh.write(txt + "\n")


if __name__ == "__main__":
    main(sys.argv[1:])
