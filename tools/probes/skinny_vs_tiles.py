"""Short-M GEMMs (CLIP text encoders at one prompt: M = 77 / 154 tokens): the skinny kernel (M <= 128, the
untuned default) against the MFMA tile kernels (v8 128x128, v10-v14 small tiles, split-K forms), in one
process, interleaved, with an fp32 check. Prints TF/s per shape.

python tools/probes/skinny_vs_tiles.py
"""
import math
import statistics
import sys

import torch

sys.path.insert(0, __file__.rsplit("/tools/", 1)[0])

from comfy_gen_server_amd import _native  # noqa: E402
from comfy_gen_server_amd.ops import core  # noqa: E402

SHAPES = [(77, 768, 768), (77, 2304, 768), (77, 3072, 768), (77, 768, 3072),            # CLIP-L
          (77, 1280, 1280), (77, 3840, 1280), (77, 5120, 1280), (77, 1280, 5120),      # CLIP-G
          (154, 3840, 1280), (154, 5120, 1280), (154, 1280, 5120), (16, 1280, 1280)]


def main():
    lib = _native.load_kernels()
    assert lib is not None, _native.kernels_error()
    dev = torch.device("cuda", 0)
    st = core._stream()
    torch.manual_seed(0)
    for M, N, K in SHAPES:
        a = torch.randn(M, K, device=dev).to(torch.bfloat16)
        w = (torch.randn(N, K, device=dev) / math.sqrt(K)).to(torch.bfloat16)
        b = torch.randn(N, device=dev).to(torch.bfloat16)
        o = torch.empty(M, N, device=dev, dtype=torch.bfloat16)
        ref = a.float() @ w.float().t() + b.float()
        cands = {}
        ws = core._skinny_ws(M, N, K, dev)

        def skinny():
            return lib.cgs_gemm_skinny_ws(a.data_ptr(), w.data_ptr(), o.data_ptr(), b.data_ptr(), None, M, N, K, K, K,
                                          N, 0, 1, 1.0, ws.data_ptr() if ws is not None else None,
                                          ws.numel() if ws is not None else 0, st)
        cands["skinny"] = skinny
        for v in (8, 10, 11, 12, 13, 14):
            cands[f"v{v}"] = (lambda v=v: lib.cgs_gemm_bf16_v(a.data_ptr(), w.data_ptr(), o.data_ptr(), b.data_ptr(),
                                                               None, M, N, K, K, K, N, 0, 1, 1.0, v, st))
        errs, times = {}, {k: [] for k in cands}
        for k, f in list(cands.items()):
            o.zero_()
            if f() != 0:
                del cands[k], times[k]
                continue
            torch.cuda.synchronize()
            errs[k] = ((o.float() - ref).abs().max() / ref.abs().max()).item()
        for _ in range(5):
            for k, f in cands.items():
                for _ in range(3):
                    f()
                torch.cuda.synchronize()
                s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                s.record()
                for _ in range(20):
                    f()
                e.record()
                torch.cuda.synchronize()
                times[k].append(s.elapsed_time(e) / 20 * 1e3)
        us = {k: statistics.median(t) for k, t in times.items()}
        best = min(us, key=us.get)
        print(f"M={M} N={N} K={K}: " + "  ".join(f"{k} {v:.1f}us" for k, v in us.items()) +
              f"  | best {best}" + (f" ({us['skinny'] / us[best]:.2f}x skinny)" if "skinny" in us else "") +
              f"  max err {max(errs.values()):.1e}", flush=True)


if __name__ == "__main__":
    main()
