"""Re-measure the packaged tuning table's GEMM entries on this GPU (after a GEMM-kernel change, e.g. new
candidates such as the split-K forms).

python -m comfy_gen_server_amd.tools.gemm_retune out.json [--m M1,M2,...] [--apply [--replace-splitk]]

Every ``gemm|M|N|K|epi`` / ``gemm_lnfold|M|N|K|epi`` key of ``data/tune_mi355x.json`` (optionally only
the listed M) is rebuilt as a random problem and run once through ``ops.linear`` / ``ops.linear_lnfold``
with the packaged table NOT loaded, so ``autotune.choose`` times every legal candidate afresh.
``out.json`` gets ``{key: {"old": ..., "choice": ..., "ms": {...}}}``; ``--apply`` also rewrites those
entries of the packaged table (run that on the development copy, not on a GPU box's snapshot). Entries that
hold a split-K choice are left alone unless ``--replace-splitk``: those were set from in-job A/Bs, and the
isolated time of a split-K launch pair disagrees with its in-job cost (round 6: the Cascade batch-1 K = 8192
projection re-timed to v14 here ran 3.9 % slower per job, profiles/r06/ab_tables_r06.log).
"""
from __future__ import annotations

import json
import os
import sys


def main(argv):
    os.environ["CGS_TUNE_DEFAULT"] = "0"
    import torch
    from comfy_gen_server_amd import ops
    from comfy_gen_server_amd.ops import autotune, core
    dev = torch.device("cuda", 0)
    with open(autotune.DEFAULT_TABLE) as f:
        table = json.load(f)
    only_m = None
    if "--m" in argv:
        only_m = {int(v) for v in argv[argv.index("--m") + 1].split(",")}
    keys = []
    for k in sorted(table):
        p = k.split("|")
        if p[0] not in ("gemm", "gemm_lnfold") or len(p) != 5:
            continue
        if only_m is not None and int(p[1]) not in only_m:
            continue
        keys.append(k)
    out = {}
    g = torch.Generator(device=dev).manual_seed(0)
    for key in keys:
        op, M, N, K, epi = key.split("|")
        M, N, K, epi = int(M), int(N), int(K), int(epi)
        x = torch.randn(M, K, device=dev, generator=g).to(torch.bfloat16)
        w = (torch.randn(N, K, device=dev, generator=g) / K ** 0.5).to(torch.bfloat16)
        b = torch.randn(N, device=dev, generator=g).to(torch.bfloat16)
        with torch.inference_mode():
            if op == "gemm":
                nout = N
                r = torch.randn(M, N, device=dev, generator=g).to(torch.bfloat16) if epi & core.EPI_RESIDUAL else None
                ops.linear(x, w, b if epi & core.EPI_BIAS else None, residual=r,
                           act="gelu" if epi & core.EPI_GELU else None)
            else:
                rs = core.layernorm_stats(x, 1e-5)
                w2, cs, b2 = core.lnfold_weights(w, b, None, None)
                core.linear_lnfold(x, rs, w2, cs, b2, geglu=bool(epi & core.EPI_GEGLU),
                                   act="gelu" if epi & core.EPI_GELU else None)
        torch.cuda.synchronize()
        ms = autotune._timings.get(key, {})
        out[key] = {"old": table[key], "choice": autotune._cache.get(key), "ms": ms}
        print(json.dumps({key: out[key]}), flush=True)
    with open(argv[0], "w") as f:
        json.dump(out, f, indent=1, sort_keys=True)
    if "--apply" in argv:
        keep_sk = "--replace-splitk" not in argv
        for k, v in out.items():
            if keep_sk and v["old"] in core._SPLITK:
                continue
            if v["choice"]:
                table[k] = v["choice"]
        with open(autotune.DEFAULT_TABLE, "w") as f:
            json.dump(table, f, indent=1, sort_keys=True)
    return 0


if __name__ == "__main__":
    sys.exit(main(sys.argv[1:]))
