"""Kernel summary of a rocprofv3 SQLite (rocpd) result: the markdown table profiles/ keeps.

    python tools/rocpd_summary.py gpurun_out/<dir>/run_results.db [--top 40] [--grids]

Per kernel name: calls, total / mean / min / max duration and share of GPU kernel time; ``--grids``
adds the most frequent (grid, workgroup) launch shape, which shows under-filled launches at small
batch (fewer workgroups than the 256 CUs).
"""
import argparse
import collections
import sqlite3


def summarize(db, top=40, grids=False):
    c = sqlite3.connect(db)
    rows = c.execute("select name, duration, grid_x, grid_y, grid_z, workgroup_x, workgroup_y, workgroup_z "
                     "from kernels").fetchall()
    agg = collections.OrderedDict()
    for name, dur, gx, gy, gz, wx, wy, wz in rows:
        a = agg.setdefault(name, {"n": 0, "t": 0, "min": None, "max": 0, "shapes": collections.Counter()})
        a["n"] += 1
        a["t"] += dur
        a["min"] = dur if a["min"] is None else min(a["min"], dur)
        a["max"] = max(a["max"], dur)
        if grids:
            wgs = (gx // max(wx, 1)) * (gy // max(wy, 1)) * (gz // max(wz, 1))
            a["shapes"][(wgs, wx * wy * wz)] += 1
    total = sum(a["t"] for a in agg.values()) or 1
    out = ["| kernel | calls | total ms | avg us | min us | max us | % |" + (" top launch (WGs x threads) |" if grids else ""),
           "|---|---:|---:|---:|---:|---:|---:|" + ("---|" if grids else "")]
    for name, a in sorted(agg.items(), key=lambda kv: -kv[1]["t"])[:top]:
        short = name if len(name) <= 90 else name[:87] + "..."
        line = (f"| `{short}` | {a['n']} | {a['t'] / 1e6:.2f} | {a['t'] / a['n'] / 1e3:.1f} | {a['min'] / 1e3:.1f} "
                f"| {a['max'] / 1e3:.1f} | {100.0 * a['t'] / total:.1f} |")
        if grids:
            (wgs, th), cnt = a["shapes"].most_common(1)[0]
            line += f" {wgs} x {th} ({cnt}) |"
        out.append(line)
    out.append("")
    out.append(f"Total GPU kernel time: {total / 1e6:.1f} ms over {sum(a['n'] for a in agg.values())} dispatches "
               f"({len(agg)} distinct kernels).")
    return "\n".join(out)


if __name__ == "__main__":
    ap = argparse.ArgumentParser()
    ap.add_argument("db")
    ap.add_argument("--top", type=int, default=40)
    ap.add_argument("--grids", action="store_true")
    a = ap.parse_args()
    print(summarize(a.db, a.top, a.grids))
