"""SDXL VAE decode timing (the headline job's decode: 8 latents of 128^2 -> 8 x 1024^2 images, bf16),
the conv FLOPs it executes and the achieved rate.

    python -m comfy_gen_server_amd.tools.vae_bench [--batch 8] [--reps 3]
"""
from __future__ import annotations

import argparse
import json
import time

import torch


def conv_flops(model, z):
    """Sum of 2 * Ho * Wo * Cin * Cout * kh * kw over the decoder's convs (forward hooks)."""
    tot = [0]
    hooks = []
    from ..models.layers import Conv2d

    def hook(m, inp, out):
        x = inp[0]
        cin = m.in_channels
        tot[0] += 2 * out.shape[0] * out.shape[2] * out.shape[3] * cin * m.out_channels * \
            m.kernel_size[0] * m.kernel_size[1]
    for mod in model.modules():
        if isinstance(mod, Conv2d):
            hooks.append(mod.register_forward_hook(hook))
    with torch.inference_mode():
        model.decode(z)
    for h in hooks:
        h.remove()
    return tot[0]


def main(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=8)
    ap.add_argument("--reps", type=int, default=3)
    ap.add_argument("--ab-gns", action="store_true",
                    help="alternate GroupNorm statistics from the conv epilogues on / off (same process)")
    a = ap.parse_args(argv)
    from ..models.layers import init_random_fast_
    from ..runtime.sd import VAE
    dev = torch.device("cuda")
    vae = VAE(sd=None, device=dev, dtype=torch.bfloat16)
    m = vae.first_stage_model.to(dev)
    init_random_fast_(m, seed=1)
    z = torch.randn(a.batch, 4, 128, 128, device=dev, dtype=torch.bfloat16)
    fl = conv_flops(m, z)
    with torch.inference_mode():
        for _ in range(2):
            m.decode(z)
        torch.cuda.synchronize()
        ts = []
        for _ in range(a.reps):
            t = time.perf_counter()
            m.decode(z)
            torch.cuda.synchronize()
            ts.append(time.perf_counter() - t)
    best = min(ts)
    print(json.dumps({"batch": a.batch, "decode_ms": round(best * 1e3, 2), "conv_tflop": round(fl / 1e12, 2),
                      "conv_tflops_per_s_upper_bound": round(fl / best / 1e12, 1)}), flush=True)
    if a.ab_gns:
        from ..ops import core
        res = {True: [], False: []}
        with torch.inference_mode():
            for _ in range(a.reps):
                for on in (True, False):
                    core._GNS = on
                    m.decode(z)
                    torch.cuda.synchronize()
                    t = time.perf_counter()
                    m.decode(z)
                    torch.cuda.synchronize()
                    res[on].append(time.perf_counter() - t)
        core._GNS = True
        print(json.dumps({"gns_on_ms": round(min(res[True]) * 1e3, 2), "gns_off_ms": round(min(res[False]) * 1e3, 2),
                          "runs_on": [round(x * 1e3, 2) for x in res[True]],
                          "runs_off": [round(x * 1e3, 2) for x in res[False]]}), flush=True)


if __name__ == "__main__":
    main()
