"""Re-measure the packaged tuning table's conv entries on this GPU (after a conv-kernel change).

python -m comfy_gen_server_amd.tools.retune out.json [--n 1,2] [--apply]

Every ``conv|...`` key of ``data/tune_mi355x.json`` is rebuilt as a real problem (shapes, dual-input
concat, nearest-2x upsample flag, residual) and run once through ``ops.conv2d`` with the packaged table
NOT loaded, so ``autotune.choose`` times every legal candidate afresh. ``out.json`` gets
``{key: {"old": ..., "choice": ..., "ms": {...}}}``; ``--apply`` also rewrites the packaged table's conv
entries with the new choices (run that on the development copy, not on a GPU box's snapshot).
"""
from __future__ import annotations

import ast
import json
import os
import sys


def _problem(key: str):
    parts = key.split("|")
    N, H, W, Cin, Cout, kh, stride, pad, flags, res = (int(v) for v in parts[1:11])
    C1 = Cin
    if len(parts) > 11:
        tag = ast.literal_eval(parts[11])
        C1 = int(tag[1])
    return N, H, W, Cin, Cout, kh, stride, pad, flags, res, C1


def main(argv):
    os.environ["CGS_TUNE_DEFAULT"] = "0"
    import torch
    from comfy_gen_server_amd.ops import autotune, core
    dev = torch.device("cuda", 0)
    with open(autotune.DEFAULT_TABLE) as f:
        table = json.load(f)
    keys = sorted(k for k in table if k.startswith("conv|"))
    if "--n" in argv:           # only the keys of these batch sizes (first key field)
        only = {int(v) for v in argv[argv.index("--n") + 1].split(",")}
        keys = [k for k in keys if int(k.split("|")[1]) in only]
    out = {}
    for key in keys:
        N, H, W, Cin, Cout, kh, stride, pad, flags, res, C1 = _problem(key)
        up = bool(flags & 16)
        Hl, Wl = (2 * H, 2 * W) if up else (H, W)
        Ho, Wo = (Hl + 2 * pad - kh) // stride + 1, (Wl + 2 * pad - kh) // stride + 1
        g = torch.Generator(device=dev).manual_seed(0)

        def rnd(*shape):
            return (torch.rand(*shape, device=dev, generator=g) * 2 - 1).to(torch.bfloat16)
        x = rnd(N, C1, H, W).contiguous(memory_format=torch.channels_last)
        x2 = rnd(N, Cin - C1, H, W).contiguous(memory_format=torch.channels_last) if C1 != Cin else None
        w = rnd(Cout, Cin, kh, kh) / (Cin * kh * kh) ** 0.5
        wn = w.permute(0, 2, 3, 1).contiguous()
        b = rnd(Cout)
        r = rnd(N, Cout, Ho, Wo).contiguous(memory_format=torch.channels_last) if res else None
        core.conv2d(x, w, b, stride, pad, residual=r, weight_nhwc=wn, upsample2x=up, x2=x2)
        torch.cuda.synchronize()
        t = autotune.table().get(key)
        if t is None:
            print(f"{key}: not re-tuned (key mismatch)", flush=True)
            continue
        out[key] = {"old": table[key], "choice": t["choice"], "ms": t.get("ms", {})}
        print(f"{key}: {table[key]} -> {t['choice']}  " +
              " ".join(f"{c}={ms:.3f}" for c, ms in sorted(t.get("ms", {}).items())), flush=True)
        del x, x2, w, wn, b, r
        torch.cuda.empty_cache()
    with open(argv[0], "w") as f:
        json.dump(out, f, indent=1, sort_keys=True)


def apply(path):
    from comfy_gen_server_amd.ops import autotune
    with open(path) as f:
        new = json.load(f)
    with open(autotune.DEFAULT_TABLE) as f:
        table = json.load(f)
    n = 0
    for k, v in new.items():
        if k in table and table[k] != v["choice"]:
            table[k] = v["choice"]
            n += 1
    with open(autotune.DEFAULT_TABLE, "w") as f:
        f.write("{\n" + ",\n".join(f"{json.dumps(k)}: {json.dumps(v)}" for k, v in table.items()) + "\n}\n")
    print(f"{n} entries changed")


if __name__ == "__main__":
    if "--apply" in sys.argv:
        apply(sys.argv[1])
    else:
        main(sys.argv[1:])
