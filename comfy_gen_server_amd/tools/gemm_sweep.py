"""Sweep GEMM variant x tile-group order on a few shapes (one process, interleaved rounds).

python -m comfy_gen_server_amd.tools.gemm_sweep [out.md]
"""
from __future__ import annotations

import math
import sys

import torch

SHAPES = [(16384, 3840, 1280), (16384, 1280, 5120), (65536, 1920, 640), (4096, 4096, 4096), (8192, 8192, 8192)]
VARIANTS = [5, 6, 7]
GROUPS = [1, 4, 8, 16]
EPI = 0
if "--kseries" in sys.argv:        # per-tile fixed cost vs per-K-tile cost: 1024 tiles (4 rounds), K swept
    SHAPES = [(16384, 4096, k) for k in (128, 256, 640, 1280, 2560, 5120)] + [(16384, 10240, 1280), (65536, 4096, 640)]
    VARIANTS = [5, 7]
    GROUPS = [8]


def main(argv):
    from comfy_gen_server_amd import _native
    from comfy_gen_server_amd.ops import core
    lib = _native.load_kernels()
    dev = torch.device("cuda", 0)
    rows = ["| M | N | K | variant | " + " | ".join(f"group {g} TF/s" for g in GROUPS) + " |",
            "|---:|---:|---:|---|" + "---:|" * len(GROUPS)]
    for M, N, K in SHAPES:
        a = (torch.rand(M, K, device=dev) * 2 - 1).to(torch.bfloat16)
        w = ((torch.rand(N, K, device=dev) * 2 - 1) / math.sqrt(K)).to(torch.bfloat16)
        out = torch.empty(M, N, device=dev, dtype=torch.bfloat16)
        res = {}
        for rnd in range(3):
            for v in VARIANTS:
                for g in GROUPS:
                    lib.cgs_set_tile_group(g)
                    fn = lambda: lib.cgs_gemm_bf16_v(a.data_ptr(), w.data_ptr(), out.data_ptr(), None, None, M, N, K,  # noqa
                                                     K, K, N, 0, EPI, 1.0, v, core._stream())
                    fn()
                    torch.cuda.synchronize()
                    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                    it = max(3, int(2e11 / (2 * M * N * K)))
                    s.record()
                    for _ in range(it):
                        fn()
                    e.record()
                    torch.cuda.synchronize()
                    ms = s.elapsed_time(e) / it
                    res.setdefault((v, g), []).append(2.0 * M * N * K / ms / 1e9)
        lib.cgs_set_tile_group(8)
        for v in VARIANTS:
            rows.append(f"| {M} | {N} | {K} | v{v} | " + " | ".join(f"{max(res[(v, g)]):.0f}" for g in GROUPS) + " |")
            print(rows[-1], flush=True)
        del a, w, out
    text = "\n".join(rows)
    argv = [a for a in argv if not a.startswith("--")]
    if argv:
        open(argv[0], "w").write(text + "\n")
    print(text)


if __name__ == "__main__":
    main(sys.argv[1:])
