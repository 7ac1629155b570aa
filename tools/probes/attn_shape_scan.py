"""Where the D = 64 attention kernel loses time at SDXL level 2: TF/s as a function of the keys per workgroup
(Sk) and the number of workgroups (B, H, Sq). If short-Sk shapes are slower at equal work, the per-workgroup
prologue / epilogue (Q load, K/V pipeline fill, O store) is not overlapped with compute."""
import os
import sys

import torch

sys.path.insert(0, os.getcwd())
from comfy_gen_server_amd.ops import core  # noqa: E402

dev = torch.device("cuda", 0)
lib = core._lib()
for B, H, Sq, Sk in [(16, 10, 4096, 4096), (16, 20, 1024, 1024), (16, 20, 1024, 4096), (16, 20, 1024, 2048),
                     (16, 20, 4096, 1024), (16, 20, 1024, 512), (16, 20, 2048, 1024), (64, 20, 1024, 1024)]:
    D = 64
    q = torch.randn(B, Sq, H * D, device=dev).to(torch.bfloat16)
    k = torch.randn(B, Sk, H * D, device=dev).to(torch.bfloat16)
    v = torch.randn(B, Sk, H * D, device=dev).to(torch.bfloat16)
    o = torch.empty_like(q)
    sq, sk = (Sq * H * D, H * D, D), (Sk * H * D, H * D, D)

    def run():
        return lib.cgs_flash_attn_fwd_v(q.data_ptr(), k.data_ptr(), v.data_ptr(), o.data_ptr(), B, H, Sq, Sk, D,
                                        *sq, *sk, *sk, *sq, D ** -0.5, 0, core._stream())
    ts = []
    for _ in range(3):
        assert run() == 0
        torch.cuda.synchronize()
        s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        s.record()
        for _ in range(20):
            run()
        e.record()
        torch.cuda.synchronize()
        ts.append(s.elapsed_time(e) / 20)
    t = sorted(ts)[1]
    fl = 4 * B * H * Sq * Sk * D
    wgs = B * H * ((Sq + 255) // 256)
    print(f"B={B} H={H} Sq={Sq} Sk={Sk}: {fl / t / 1e9:.0f} TF/s ({t * 1e3:.1f} us)  WGs={wgs} "
          f"({wgs / 256:.2f} rounds)  us/WG-round={t * 1e3 / (wgs / 256):.2f}", flush=True)
