"""GroupNorm (+ SiLU) time on the SDXL UNet / VAE shapes through cgs_groupnorm_nhwc_ws (statistics pass,
finalize and apply), checked against torch.group_norm + silu in fp32; CGS_LIB=<other libcgs_kernels.so> runs
another build (library A/B, one process per build).

python tools/probes/gn_apply_ab.py"""
import os
import sys

import torch

sys.path.insert(0, os.getcwd())
from comfy_gen_server_amd.ops import core  # noqa: E402

dev = torch.device("cuda", 0)
if os.environ.get("CGS_LIB"):
    from comfy_gen_server_amd.tools.ab_bench import _use_lib
    _use_lib(os.environ["CGS_LIB"])
lib = core._lib()
torch.manual_seed(0)
tot = 0.0
for N, H, C in [(16, 128, 320), (16, 128, 960), (16, 64, 640), (16, 64, 1920), (16, 32, 1280), (16, 32, 2560),
                (8, 1024, 128), (8, 512, 256), (8, 256, 512)]:
    HW = H * H
    x = torch.randn(N, HW, C, device=dev).to(torch.bfloat16)
    y = torch.empty_like(x)
    g = (1 + 0.1 * torch.randn(C, device=dev)).to(torch.bfloat16)
    b = (0.1 * torch.randn(C, device=dev)).to(torch.bfloat16)
    ws = torch.empty(int(lib.cgs_groupnorm_workspace(N, HW, C)), dtype=torch.uint8, device=dev)

    def run():
        return lib.cgs_groupnorm_nhwc_ws(x.data_ptr(), y.data_ptr(), g.data_ptr(), b.data_ptr(), None, ws.data_ptr(),
                                         N, HW, C, 32, 1e-5, 1, 1, core._stream())
    ts = []
    for _ in range(5):
        assert run() == 0
        torch.cuda.synchronize()
        s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        s.record()
        for _ in range(10):
            run()
        e.record()
        torch.cuda.synchronize()
        ts.append(s.elapsed_time(e) / 10)
    t = sorted(ts)[2]
    tot += t
    xs = x[:2].float().permute(0, 2, 1).reshape(2, C, H, H)
    ref = torch.nn.functional.silu(torch.nn.functional.group_norm(xs, 32, g.float(), b.float(), 1e-5))
    err = (y[:2].float().permute(0, 2, 1).reshape(2, C, H, H) - ref).abs().max().item()
    gb = 3 * x.numel() * 2 / 1e9
    print(f"lib={os.environ.get('CGS_LIB', 'in-tree')} N={N} {H}x{H} C={C}: {t * 1e3:.1f} us "
          f"({gb / t:.2f} TB/s of 2 reads + 1 write)  max|y-fp32|={err:.4f}", flush=True)
    assert err < 0.05, err
    del x, y, ws
print(f"lib={os.environ.get('CGS_LIB', 'in-tree')} total {tot * 1e3:.1f} us", flush=True)
