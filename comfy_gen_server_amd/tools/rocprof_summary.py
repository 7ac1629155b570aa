"""Summarise a rocprofv3 ``--kernel-trace`` database into a per-kernel stats table (markdown).

Usage: python -m comfy_gen_server_amd.tools.rocprof_summary gpurun_out/prof/run_results.db [out.md] [--top N]
       [--tail-s S]  (only the last S seconds of the trace)
Kernel names are demangled-ish (template args beyond the first are cut) so CK / MIOpen / our own
kernels are readable side by side.
"""
from __future__ import annotations

import re
import sqlite3
import sys


def short_name(name: str, width: int = 90) -> str:
    n = name
    if n.startswith("_ZN"):   # mangled (CK / Tensile): keep the readable identifier chunks
        parts = re.findall(r"\d+([A-Za-z_][A-Za-z0-9_]*)", n[:400])
        n = "::".join(p for p in parts[:6] if len(p) > 2)
    n = n.replace("(anonymous namespace)", "anon")
    n = re.sub(r"\(.*", "", n)
    return n if len(n) <= width else n[: width - 3] + "..."


def summarize(db: str, top: int = 40, tail_s: float | None = None):
    """``tail_s``: only kernels that start in the last ``tail_s`` seconds of the trace (steady state:
    drops the warmup / autotune trials at the front)."""
    c = sqlite3.connect(db)
    where = ""
    if tail_s:
        t_end = c.execute("select max(end) from kernels").fetchone()[0]
        where = f" where start >= {int(t_end - tail_s * 1e9)}"
    rows = list(c.execute("select name, count(*), sum(duration), avg(duration), min(duration), max(duration) "
                          f"from kernels{where} group by name order by sum(duration) desc"))
    total = sum(r[2] for r in rows) or 1
    out = ["| kernel | calls | total ms | avg us | min us | max us | % |", "|---|---:|---:|---:|---:|---:|---:|"]
    for name, n, tot, avg, mn, mx in rows[:top]:
        out.append(f"| `{short_name(name)}` | {n} | {tot / 1e6:.2f} | {avg / 1e3:.1f} | {mn / 1e3:.1f} | "
                   f"{mx / 1e3:.1f} | {100.0 * tot / total:.1f} |")
    out.append(f"\nTotal GPU kernel time: {total / 1e6:.1f} ms over {sum(r[1] for r in rows)} dispatches "
               f"({len(rows)} distinct kernels).")
    return "\n".join(out)


def main(argv):
    top = 40
    if "--top" in argv:
        i = argv.index("--top")
        top = int(argv[i + 1])
        argv = argv[:i] + argv[i + 2:]
    tail = None
    if "--tail-s" in argv:
        i = argv.index("--tail-s")
        tail = float(argv[i + 1])
        argv = argv[:i] + argv[i + 2:]
    text = summarize(argv[0], top, tail)
    if len(argv) > 1:
        with open(argv[1], "w") as f:
            f.write(text + "\n")
    print(text)


if __name__ == "__main__":
    main(sys.argv[1:])
