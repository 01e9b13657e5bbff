"""Summarise rocprofv3 --pmc databases: per kernel (short name), the mean over dispatches of each counter
(summed over its instances within a dispatch) and the mean dispatch duration.

usage: python tools/pmc_summary.py DB [DB ...] [--filter SUBSTR]"""
import re
import sqlite3
import sys
from collections import defaultdict

sys.path.insert(0, __file__.rsplit("/", 1)[0])
from prof_summary import short  # noqa: E402


def main():
    args = sys.argv[1:]
    filt = None
    if "--filter" in args:
        i = args.index("--filter")
        filt = args[i + 1]
        del args[i:i + 2]
    out = defaultdict(lambda: defaultdict(list))
    dur = defaultdict(dict)
    for db in args:
        c = sqlite3.connect(db)
        per = defaultdict(float)
        for name, disp, cname, val, d in c.execute(
                "select name, dispatch_id, counter_name, counter_value, duration from pmc_events"):
            k = short(name)
            if filt and filt not in k:
                continue
            per[(k, disp, cname)] += val
            dur[k][(db, disp)] = d
        for (k, disp, cname), v in per.items():
            out[k][cname].append(v)
    for k in sorted(out, key=lambda k: -sum(dur[k].values())):
        ds = list(dur[k].values())
        print(f"{k}  dispatches={len(ds)} mean_us={sum(ds) / len(ds) / 1e3:.1f}")
        for cname in sorted(out[k]):
            vs = out[k][cname]
            print(f"    {cname:32s} {sum(vs) / len(vs):.4g}")


if __name__ == "__main__":
    main()
