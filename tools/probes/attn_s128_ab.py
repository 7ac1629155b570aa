"""In-process A/B of the 128-key LDS stages for the 8-wave D = 64 attention kernel (round 6, NOT adopted:
-11 % at level 1, -2 % per job; profiles/r06/attn_s128_*.log). Needs profiles/r06/attn_s128_experiment.patch
applied (it adds cgs_attn_set_s128). Outputs must be bitwise equal and match an fp32 reference."""
import os
import sys

import torch

sys.path.insert(0, os.getcwd())
from comfy_gen_server_amd.ops import core  # noqa: E402

dev = torch.device("cuda", 0)
lib = core._lib()
torch.manual_seed(0)
for B, H, Sq, Sk in [(16, 10, 4096, 4096), (16, 20, 1024, 1024), (2, 20, 1024, 1024), (2, 10, 4096, 4096),
                     (4, 10, 1024, 960), (4, 10, 1024, 1000), (4, 10, 512, 64), (4, 10, 512, 100),
                     (4, 10, 512, 4160), (1, 2, 300, 193)]:
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
            lib.cgs_attn_set_s128(t)
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
    lib.cgs_attn_set_s128(0)
    qh = q.float().view(B, Sq, H, D).transpose(1, 2)
    kh = k.float().view(B, Sk, H, D).transpose(1, 2)
    vh = v.float().view(B, Sk, H, D).transpose(1, 2)
    ref = torch.nn.functional.scaled_dot_product_attention(qh, kh, vh).transpose(1, 2).reshape(B, Sq, H * D)
    err = (outs[1].float() - ref).abs().max().item()
    fl = 4 * B * H * Sq * Sk * D
    line = "  ".join(f"s128={t}: {fl / sorted(v)[1] / 1e9:.0f} TF/s ({sorted(v)[1] * 1e3:.1f} us)"
                     for t, v in res.items())
    print(f"B={B} H={H} Sq={Sq} Sk={Sk}: {line}  bitwise-equal={torch.equal(outs[0], outs[1])}  "
          f"max|s128-fp32|={err:.4f}", flush=True)
    assert err < 0.02, err
