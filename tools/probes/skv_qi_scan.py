"""Short-KV cross-attention (K03) time at the SDXL shapes for the QI setting of this process (CGS_SKV_QI=1|2|4,
read once per process), checked against an fp32 reference. Run once per setting:

for q in 1 2 4; do CGS_SKV_QI=$q python tools/probes/skv_qi_scan.py; done"""
import os
import sys

import torch

sys.path.insert(0, os.getcwd())
from comfy_gen_server_amd.ops import core  # noqa: E402

dev = torch.device("cuda", 0)
if os.environ.get("CGS_LIB"):     # another build of libcgs_kernels.so (library A/B)
    from comfy_gen_server_amd.tools.ab_bench import _use_lib
    _use_lib(os.environ["CGS_LIB"])
lib = core._lib()
torch.manual_seed(0)
for B, H, Sq, Sk in [(16, 20, 1024, 77), (16, 10, 4096, 77), (2, 20, 1024, 77), (2, 10, 4096, 77)]:
    D = 64
    q = torch.randn(B, Sq, H * D, device=dev).to(torch.bfloat16)
    k = torch.randn(B, Sk, H * D, device=dev).to(torch.bfloat16)
    v = torch.randn(B, Sk, H * D, device=dev).to(torch.bfloat16)
    o = torch.empty_like(q)
    sq, sk = (Sq * H * D, H * D, D), (Sk * H * D, H * D, D)

    def run():
        return lib.cgs_flash_attn_fwd_v(q.data_ptr(), k.data_ptr(), v.data_ptr(), o.data_ptr(), B, H, Sq, Sk, D,
                                        *sq, *sk, *sk, *sq, D ** -0.5, 3, core._stream())
    ts = []
    for _ in range(5):
        assert run() == 0
        torch.cuda.synchronize()
        s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        s.record()
        for _ in range(50):
            run()
        e.record()
        torch.cuda.synchronize()
        ts.append(s.elapsed_time(e) / 50)
    qh = q.float().view(B, Sq, H, D).transpose(1, 2)
    kh = k.float().view(B, Sk, H, D).transpose(1, 2)
    vh = v.float().view(B, Sk, H, D).transpose(1, 2)
    ref = torch.nn.functional.scaled_dot_product_attention(qh, kh, vh).transpose(1, 2).reshape(B, Sq, H * D)
    err = (o.float() - ref).abs().max().item()
    t = sorted(ts)[2]
    gb = 2 * q.numel() * 2 / 1e9
    print(f"QI={os.environ.get('CGS_SKV_QI', 'auto')} lib={os.environ.get('CGS_LIB', 'in-tree')} B={B} H={H} Sq={Sq} Sk={Sk}: {t * 1e3:.1f} us "
          f"({gb / t:.2f} TB/s of Q + O)  max|out-fp32|={err:.4f}", flush=True)
    assert err < 0.02, err
