"""In-process A/B: LayerNorm-folded GEGLU on v6 (256x160, pq::run GG) vs v7 (256x256) on the SDXL shapes
(batch 8: M = 16384 / 65536; batch 1: M = 2048 / 8192), median of 3 interleaved rounds."""
import math
import os
import sys

import torch

sys.path.insert(0, os.getcwd())
from comfy_gen_server_amd import _native  # noqa: E402
from comfy_gen_server_amd.ops import core  # noqa: E402

lib = _native.load_kernels()
dev = torch.device("cuda", 0)
for M, N2, K in [(16384, 10240, 1280), (65536, 5120, 640), (2048, 10240, 1280), (8192, 5120, 640), (4096, 10240, 1280)]:
    a = torch.randn(M, K, device=dev).to(torch.bfloat16)
    w = (torch.randn(N2, K, device=dev) / math.sqrt(K)).to(torch.bfloat16)
    b = torch.randn(N2, device=dev).to(torch.bfloat16)
    rs = core.layernorm_stats(a, 1e-5)
    cs = w.float().sum(dim=1).contiguous()
    out = torch.empty(M, N2 // 2, device=dev, dtype=torch.bfloat16)
    ws = core._v7_ws(M, N2, K, dev)

    def run(v):
        return lib.cgs_gemm_bf16_lnfold_v(a.data_ptr(), w.data_ptr(), out.data_ptr(), b.data_ptr(), rs.data_ptr(),
                                          cs.data_ptr(), M, N2, K, K, K, N2 // 2, core.EPI_BIAS | core.EPI_GEGLU,
                                          None if ws is None or v != 7 else ws.data_ptr(),
                                          0 if ws is None or v != 7 else ws.numel(), v, core._stream())
    res = {6: [], 7: []}
    for _ in range(3):
        for v in (6, 7):
            assert run(v) == 0
            torch.cuda.synchronize()
            s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            s.record()
            for _ in range(20):
                run(v)
            e.record()
            torch.cuda.synchronize()
            res[v].append(s.elapsed_time(e) / 20)
    outs = {}
    for v in (6, 7):
        run(v)
        torch.cuda.synchronize()
        outs[v] = out.float().clone()
    d = ((outs[6] - outs[7]).norm() / outs[7].norm()).item()
    print(f"ln:geglu M={M} N2={N2} K={K}: " + " ".join(
        f"v{v}={2 * M * N2 * K / sorted(t)[1] / 1e9:.0f} TF/s ({sorted(t)[1] * 1e3:.0f} us)" for v, t in res.items()) +
        f" rel(v6, v7)={d:.1e}", flush=True)
    del a, w, out, ws
