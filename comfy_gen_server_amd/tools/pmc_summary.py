"""Summarise rocprofv3 ``--pmc`` databases: mean counter value per dispatch for kernels whose name
matches a pattern, plus derived rates (MFMA busy %, LDS bank-conflict ratio, L2 hit rate).

python -m comfy_gen_server_amd.tools.pmc_summary <pattern> db1 [db2 ...]
"""
from __future__ import annotations

import collections
import sqlite3
import sys


def collect(db, pattern):
    c = sqlite3.connect(db)
    rows = c.execute("select kernel_name, counter_name, value, duration, dispatch_id from counters_collection "
                     "where kernel_name like ?", (f"%{pattern}%",))
    per = collections.defaultdict(list)
    durs = {}
    for name, cn, v, dur, did in rows:
        per[cn].append(v)
        durs[did] = dur
    return {k: sum(v) / len(v) for k, v in per.items()}, (sum(durs.values()) / len(durs) if durs else 0.0), len(durs)


def main(argv):
    pat, dbs = argv[0], argv[1:]
    for db in dbs:
        vals, dur, n = collect(db, pat)
        print(f"== {db}: {n} dispatches, mean {dur / 1e3:.1f} us")
        for k in sorted(vals):
            print(f"   {k:32s} {vals[k]:.4g}")
        if "SQ_VALU_MFMA_BUSY_CYCLES" in vals and "SQ_BUSY_CYCLES" in vals and vals["SQ_BUSY_CYCLES"]:
            print(f"   -> MFMA busy / SQ busy       {vals['SQ_VALU_MFMA_BUSY_CYCLES'] / vals['SQ_BUSY_CYCLES']:.3f}")
        if "SQ_LDS_BANK_CONFLICT" in vals and vals.get("SQ_LDS_IDX_ACTIVE"):
            print(f"   -> LDS conflict / active     {vals['SQ_LDS_BANK_CONFLICT'] / vals['SQ_LDS_IDX_ACTIVE']:.3f}")
        if "TCC_HIT_sum" in vals and "TCC_MISS_sum" in vals:
            tot = vals["TCC_HIT_sum"] + vals["TCC_MISS_sum"]
            print(f"   -> L2 hit rate               {vals['TCC_HIT_sum'] / tot if tot else 0:.3f}")


if __name__ == "__main__":
    main(sys.argv[1:])
