"""Idle time of the GPU between kernels in a rocprofv3 ``--kernel-trace`` database: the union of all
kernel intervals (every stream) over the traced window, the total idle time, and the largest idle gaps
with the kernels on either side -- where a job still waits on the host (sampler bookkeeping, CLIP, VAE
hand-off, gathers).

Usage: python -m comfy_gen_server_amd.tools.rocprof_gaps run_results.db [--tail-s S] [--top N] [--min-us U]
"""
from __future__ import annotations

import sqlite3
import sys
from collections import defaultdict

from .rocprof_summary import short_name


def gaps(db: str, tail_s: float | None = None, top: int = 25, min_us: float = 20.0) -> str:
    c = sqlite3.connect(db)
    rows = list(c.execute("select start, end, name from kernels order by start"))
    if not rows:
        return "no kernels"
    t_end = max(r[1] for r in rows)
    t0 = t_end - int(tail_s * 1e9) if tail_s else rows[0][0]
    rows = [r for r in rows if r[1] > t0]
    busy, idle, cur_end, prev = 0, [], None, None
    for s, e, n in rows:
        s = max(s, t0)
        if cur_end is None:
            cur_end, prev = e, n
            busy += e - s
            continue
        if s > cur_end:
            idle.append((s - cur_end, prev, n))
            busy += e - s
            cur_end, prev = e, n
        elif e > cur_end:
            busy += e - cur_end
            cur_end, prev = e, n
    window = cur_end - max(t0, rows[0][0])
    tot_idle = sum(g for g, _, _ in idle)
    big = [g for g in idle if g[0] >= min_us * 1e3]
    by_pair = defaultdict(lambda: [0, 0])
    for g, a, b in big:
        k = (short_name(a, 60), short_name(b, 60))
        by_pair[k][0] += g
        by_pair[k][1] += 1
    out = [f"window {window / 1e6:.1f} ms, kernels busy {busy / 1e6:.1f} ms ({100 * busy / window:.1f} %), "
           f"idle {tot_idle / 1e6:.1f} ms in {len(idle)} gaps; {len(big)} gaps >= {min_us:.0f} us total "
           f"{sum(g for g, _, _ in big) / 1e6:.1f} ms", "",
           "| idle ms | gaps | after kernel | before kernel |", "|---:|---:|---|---|"]
    for (a, b), (g, n) in sorted(by_pair.items(), key=lambda kv: -kv[1][0])[:top]:
        out.append(f"| {g / 1e6:.2f} | {n} | `{a}` | `{b}` |")
    return "\n".join(out)


def main(argv):
    tail = top = None
    min_us = 20.0
    if "--tail-s" in argv:
        i = argv.index("--tail-s")
        tail = float(argv[i + 1])
        argv = argv[:i] + argv[i + 2:]
    if "--top" in argv:
        i = argv.index("--top")
        top = int(argv[i + 1])
        argv = argv[:i] + argv[i + 2:]
    if "--min-us" in argv:
        i = argv.index("--min-us")
        min_us = float(argv[i + 1])
        argv = argv[:i] + argv[i + 2:]
    print(gaps(argv[0], tail, top or 25, min_us))


if __name__ == "__main__":
    main(sys.argv[1:])
