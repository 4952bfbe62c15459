"""Summarise a rocprofv3 --pmc rocpd database: per kernel (name substring filter), mean counter
value per dispatch and mean duration. usage: python tools/pmc_summary.py <db> [name_filter]"""
import sqlite3
import sys
from collections import defaultdict


def summarise(db, filt="gemm_kernel"):
    c = sqlite3.connect(db)
    rows = c.execute("select dispatch_id, kernel_name, counter_name, sum(value), max(end-start) "
                     "from counters_collection group by dispatch_id, counter_name").fetchall()
    agg = defaultdict(lambda: defaultdict(list))
    dur = defaultdict(dict)
    for did, name, cn, v, d in rows:
        if filt not in name:
            continue
        short = name.replace("(anonymous namespace)::", "").split("(")[0][-90:]
        agg[short][cn].append(v)
        dur[short][did] = d
    out = {}
    for k, cs in agg.items():
        out[k] = {cn: sum(v) / len(v) for cn, v in cs.items()}
        out[k]["dispatches"] = len(dur[k])
        out[k]["mean_ns"] = sum(dur[k].values()) / len(dur[k])
    return out


if __name__ == "__main__":
    res = summarise(sys.argv[1], sys.argv[2] if len(sys.argv) > 2 else "gemm_kernel")
    for k, v in res.items():
        print(k)
        for cn, x in sorted(v.items()):
            print(f"   {cn:28s} {x:.4g}")
