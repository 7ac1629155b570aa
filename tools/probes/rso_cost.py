"""What the row-statistics epilogue (pq::run RSO: per-row LayerNorm partials of the stored outputs) costs the v6 GEMM
on the SDXL headline residual shapes: cgs_gemm_bf16_v variant 6 vs cgs_gemm_bf16_rowstats (same operands), plus the
combine launch (cgs_ln_rs_from_partials) and the statistics pass it replaces (cgs_layernorm_stats); one process,
interleaved, median of 5."""
import os
import statistics
import sys

import torch

sys.path.insert(0, os.getcwd())
from comfy_gen_server_amd.ops import core  # noqa: E402

dev = torch.device("cuda", 0)
lib = core._lib()
s = core._stream()


def _t(f, n=20):
    f()
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(n):
        f()
    b.record()
    torch.cuda.synchronize()
    return a.elapsed_time(b) / n * 1e3


for name, M, N, K in [("out1280+res", 16384, 1280, 1280), ("ffout1280+res", 16384, 1280, 5120),
                      ("out640+res", 65536, 640, 640), ("ffout640+res", 65536, 640, 2560)]:
    a = torch.randn(M, K, device=dev).to(torch.bfloat16)
    w = (torch.randn(N, K, device=dev) / K ** 0.5).to(torch.bfloat16)
    b = torch.randn(N, device=dev).to(torch.bfloat16)
    r = torch.randn(M, N, device=dev).to(torch.bfloat16)
    y = torch.empty(M, N, device=dev, dtype=torch.bfloat16)
    part = torch.empty(M, N // 80, 2, device=dev, dtype=torch.float32)
    rs = torch.empty(M, 2, device=dev, dtype=torch.float32)

    def plain():
        assert lib.cgs_gemm_bf16_v(a.data_ptr(), w.data_ptr(), y.data_ptr(), b.data_ptr(), r.data_ptr(), M, N, K, K, K,
                                   N, N, 3, 1.0, 6, s) == 0

    def rso():
        assert lib.cgs_gemm_bf16_rowstats(a.data_ptr(), w.data_ptr(), y.data_ptr(), b.data_ptr(), r.data_ptr(), M, N,
                                          K, K, K, N, N, 3, 1.0, part.data_ptr(), s) == 0

    def combine():
        assert lib.cgs_ln_rs_from_partials(part.data_ptr(), rs.data_ptr(), M, N // 80, 1e-5, s) == 0

    def stats():
        assert lib.cgs_layernorm_stats(y.data_ptr(), rs.data_ptr(), M, N, 1e-5, 1, s) == 0
    ts = {"plain": [], "rso": [], "combine": [], "stats": []}
    for _ in range(5):
        for k, f in (("plain", plain), ("rso", rso), ("combine", combine), ("stats", stats)):
            ts[k].append(_t(f))
    m = {k: statistics.median(v) for k, v in ts.items()}
    print(f"{name}: v6 {m['plain']:.1f} us, v6+RSO {m['rso']:.1f} us ({m['rso'] / m['plain'] - 1:+.1%}), combine "
          f"{m['combine']:.1f} us, statistics pass {m['stats']:.1f} us -> RSO path {m['rso'] + m['combine']:.1f} vs "
          f"plain + pass {m['plain'] + m['stats']:.1f} us", flush=True)
