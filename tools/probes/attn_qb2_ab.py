"""In-process A/B of the D = 64 attention forms by variant (cgs_flash_attn_fwd_v): 2 = 8 waves x 32 rows,
5 = 4 waves x 32 rows (two WGs per CU), 6 = 4 waves x two 32-row q-blocks (attn_fwd_d64_qb2_kernel, needs
profiles/r06/attn_qb2_experiment.patch applied), on the SDXL shapes plus odd tile / row counts; every output is
checked against an fp32 reference.

python tools/probes/attn_qb2_ab.py [variants, default 2,6]"""
import os
import sys

import torch

sys.path.insert(0, os.getcwd())
from comfy_gen_server_amd.ops import core  # noqa: E402

dev = torch.device("cuda", 0)
lib = core._lib()
VARS = [int(v) for v in (sys.argv[1] if len(sys.argv) > 1 else '2,6').split(',')]
torch.manual_seed(0)
for B, H, Sq, Sk in [(16, 10, 4096, 4096), (16, 20, 1024, 1024), (2, 20, 1024, 1024), (2, 10, 4096, 4096),
                     (4, 10, 1024, 960), (4, 10, 1000, 1000), (4, 10, 512, 64), (4, 10, 300, 100),
                     (4, 10, 512, 4160), (1, 2, 300, 193)]:
    D = 64
    q = torch.randn(B, Sq, H * D, device=dev).to(torch.bfloat16)
    k = torch.randn(B, Sk, H * D, device=dev).to(torch.bfloat16)
    v = torch.randn(B, Sk, H * D, device=dev).to(torch.bfloat16)
    o = torch.empty_like(q)
    sq, sk = (Sq * H * D, H * D, D), (Sk * H * D, H * D, D)

    def run(var):
        return lib.cgs_flash_attn_fwd_v(q.data_ptr(), k.data_ptr(), v.data_ptr(), o.data_ptr(), B, H, Sq, Sk, D,
                                        *sq, *sk, *sk, *sq, D ** -0.5, var, core._stream())
    res = {t: [] for t in VARS}
    outs = {}
    for _ in range(3):
        for t in VARS:
            assert run(t) == 0
            torch.cuda.synchronize()
            s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            s.record()
            for _ in range(20):
                run(t)
            e.record()
            torch.cuda.synchronize()
            res[t].append(s.elapsed_time(e) / 20)
            outs[t] = o.clone()
    qh = q.float().view(B, Sq, H, D).transpose(1, 2)
    kh = k.float().view(B, Sk, H, D).transpose(1, 2)
    vh = v.float().view(B, Sk, H, D).transpose(1, 2)
    ref = torch.nn.functional.scaled_dot_product_attention(qh, kh, vh).transpose(1, 2).reshape(B, Sq, H * D)
    errs = {t: (outs[t].float() - ref).abs().max().item() for t in VARS}
    fl = 4 * B * H * Sq * Sk * D
    line = "  ".join(f"v{t}: {fl / sorted(v)[1] / 1e9:.0f} TF/s ({sorted(v)[1] * 1e3:.1f} us, err {errs[t]:.4f})"
                     for t, v in res.items())
    print(f"B={B} H={H} Sq={Sq} Sk={Sk}: {line}", flush=True)
    assert max(errs.values()) < 0.02, errs
