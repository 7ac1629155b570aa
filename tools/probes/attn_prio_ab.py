"""In-process A/B on the SDXL attention shapes (bitwise-equal outputs required): first used for the 16-B
O stores (T21, kept), now for s_setprio around the P.V MFMAs (cgs_attn_set_prio)."""
import os
import sys

import torch

sys.path.insert(0, os.getcwd())
from comfy_gen_server_amd.ops import core  # noqa: E402

dev = torch.device("cuda", 0)
lib = core._lib()
for B, H, Sq, Sk in [(16, 10, 4096, 4096), (16, 20, 1024, 1024), (16, 10, 4096, 77), (16, 20, 1024, 77),
                     (2, 20, 1024, 1024), (2, 10, 4096, 77)]:
    D = 64
    q = torch.randn(B, Sq, H * D, device=dev).to(torch.bfloat16)
    k = torch.randn(B, Sk, H * D, device=dev).to(torch.bfloat16)
    v = torch.randn(B, Sk, H * D, device=dev).to(torch.bfloat16)
    o = torch.empty_like(q)
    sq, sk = (Sq * H * D, H * D, D), (Sk * H * D, H * D, D)

    def run():
        return lib.cgs_flash_attn_fwd_v(q.data_ptr(), k.data_ptr(), v.data_ptr(), o.data_ptr(), B, H, Sq, Sk, D,
                                        *sq, *sk, *sk, *sq, D ** -0.5, 0, core._stream())
    res = {0: [], 1: []}
    outs = {}
    for _ in range(3):
        for t in (0, 1):
            lib.cgs_attn_set_prio(t)
            assert run() == 0
            torch.cuda.synchronize()
            s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            s.record()
            for _ in range(20):
                run()
            e.record()
            torch.cuda.synchronize()
            res[t].append(s.elapsed_time(e) / 20)
            outs[t] = o.clone()
    lib.cgs_attn_set_prio(0)
    fl = 4 * B * H * Sq * Sk * D
    line = "  ".join(f"prio={t}: {fl / sorted(v)[1] / 1e9:.0f} TF/s ({sorted(v)[1] * 1e3:.1f} us)" for t, v in res.items())
    print(f"B={B} H={H} Sq={Sq} Sk={Sk}: {line}  bitwise-equal={torch.equal(outs[0], outs[1])}", flush=True)
