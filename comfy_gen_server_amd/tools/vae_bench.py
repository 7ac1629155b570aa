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


def layer_table(model, z):
    """One decode with CUDA events around every Conv2d / GroupNorm / AttnBlock forward: per-module time (ms), the
    conv FLOP rate, and the share of the decode, largest first (events serialise nothing: one stream)."""
    from ..models.layers import Conv2d, GroupNorm
    from ..models.vae import AttnBlock
    rec = []
    hooks = []

    def pre(mod, inp):
        ev = torch.cuda.Event(enable_timing=True)
        ev.record()
        mod._cgs_ev = ev

    def post(mod, inp, out):
        ev = torch.cuda.Event(enable_timing=True)
        ev.record()
        x = inp[0]
        fl = 0
        if isinstance(mod, Conv2d):
            fl = 2 * out.shape[0] * out.shape[2] * out.shape[3] * mod.in_channels * mod.out_channels * \
                mod.kernel_size[0] * mod.kernel_size[1]
        rec.append((mod._cgs_name, type(mod).__name__, tuple(x.shape), tuple(out.shape), fl, mod._cgs_ev, ev))
    for name, mod in model.decoder.named_modules():
        if isinstance(mod, (Conv2d, GroupNorm, AttnBlock)):
            mod._cgs_name = name
            hooks += [mod.register_forward_pre_hook(pre), mod.register_forward_hook(post)]
    with torch.inference_mode():
        t0 = torch.cuda.Event(enable_timing=True)
        t1 = torch.cuda.Event(enable_timing=True)
        t0.record()
        model.decode(z)
        t1.record()
    torch.cuda.synchronize()
    for h in hooks:
        h.remove()
    tot = t0.elapsed_time(t1)
    rows = []
    for name, kind, si, so, fl, e0, e1 in rec:
        ms = e0.elapsed_time(e1)
        rows.append((ms, name, kind, si, so, fl))
    rows.sort(key=lambda r: -r[0])
    by_kind = {}
    for ms, name, kind, si, so, fl in rows:
        by_kind[kind] = by_kind.get(kind, 0.0) + ms
    print(f"decode {tot:.2f} ms; by module kind: " + ", ".join(f"{k} {v:.2f} ms" for k, v in by_kind.items()))
    print("| module | kind | in | out | ms | TF/s | % |")
    print("|---|---|---|---|---:|---:|---:|")
    for ms, name, kind, si, so, fl in rows:
        tf = f"{fl / ms / 1e9:.0f}" if fl else ""
        print(f"| {name} | {kind} | {list(si)} | {list(so)} | {ms:.3f} | {tf} | {100 * ms / tot:.1f} |", flush=True)


def main(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=8)
    ap.add_argument("--reps", type=int, default=3)
    ap.add_argument("--layers", action="store_true",
                    help="per-module GPU time of one decode (CUDA events around every Conv2d / GroupNorm / AttnBlock)")
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
    if a.layers:
        layer_table(m, z)
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
