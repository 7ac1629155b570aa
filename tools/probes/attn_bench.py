"""D=64 attention kernel timing on the SDXL shapes (bench batch 8 x CFG 2 = 16, and batch 1 = 2):
TF/s = 4 * B * H * Sq * Sk * D / time, median of 3 x 20 launches, for kernel variants 2 (256-row Q
blocks, 8 waves) and 5 (128-row, 4 waves)."""
import os
import sys

import torch

sys.path.insert(0, os.getcwd())
from comfy_gen_server_amd.ops import core  # noqa: E402

dev = torch.device("cuda", 0)
lib = core._lib()
for B, H, S in [(16, 10, 4096), (16, 20, 1024), (2, 10, 4096), (2, 20, 1024)]:
    D = 64
    q = torch.randn(B, S, H * D, device=dev).to(torch.bfloat16)
    k = torch.randn(B, S, H * D, device=dev).to(torch.bfloat16)
    v = torch.randn(B, S, H * D, device=dev).to(torch.bfloat16)
    o = torch.empty_like(q)
    st = (S * H * D, H * D, D)
    cols = []
    for var in (2, 5):
        def run():
            return lib.cgs_flash_attn_fwd_v(q.data_ptr(), k.data_ptr(), v.data_ptr(), o.data_ptr(), B, H, S, S, D,
                                            *st, *st, *st, *st, D ** -0.5, var, core._stream())
        assert run() == 0
        ts = []
        for _ in range(3):
            torch.cuda.synchronize()
            s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            s.record()
            for _ in range(20):
                run()
            e.record()
            torch.cuda.synchronize()
            ts.append(s.elapsed_time(e) / 20)
        ms = sorted(ts)[1]
        cols.append(f"v{var}={4 * B * H * S * S * D / ms / 1e9:.0f} TF/s ({ms * 1e3:.0f} us)")
    print(f"B={B} H={H} S={S}: " + "  ".join(cols), flush=True)
