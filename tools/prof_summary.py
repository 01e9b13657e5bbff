"""Summarise a rocprofv3 kernel-trace database (rocpd SQLite) into a per-kernel CSV.

usage: python tools/prof_summary.py gpurun_out/prof/run_results.db [out.csv] [--top N]
Kernel names are shortened to the template head (argument lists dropped).
"""
import csv
import re
import sqlite3
import sys
from collections import defaultdict


def short(name: str) -> str:
    name = re.sub(r"^void ", "", name)
    depth, out = 0, []
    for ch in name:  # drop the (...) argument list, keep template args
        if ch == "(" and depth == 0 and out and not "".join(out).endswith("anonymous namespace"):
            if "".join(out).rstrip().endswith("operator"):
                out.append(ch)
                continue
            break
        out.append(ch)
    s = "".join(out).replace("(anonymous namespace)::", "")
    return s[:160]


def main():
    db = sys.argv[1]
    out = sys.argv[2] if len(sys.argv) > 2 and not sys.argv[2].startswith("--") else None
    top = int(sys.argv[sys.argv.index("--top") + 1]) if "--top" in sys.argv else 40
    c = sqlite3.connect(db)
    agg = defaultdict(lambda: [0, 0, 1 << 62, 0, ""])
    for name, dur, gx, wx in c.execute("select name, duration, grid_x, workgroup_x from kernels"):
        k = short(name)
        a = agg[k]
        a[0] += 1
        a[1] += dur
        a[2] = min(a[2], dur)
        a[3] = max(a[3], dur)
        a[4] = f"{gx // max(wx, 1)}x{wx}"
    total = sum(a[1] for a in agg.values())
    rows = sorted(agg.items(), key=lambda kv: -kv[1][1])
    w = csv.writer(open(out, "w", newline="") if out else sys.stdout)
    w.writerow(["kernel", "calls", "total_us", "avg_us", "min_us", "max_us", "pct", "last_grid"])
    for k, (n, t, mn, mx, g) in rows[:top]:
        w.writerow([k, n, f"{t / 1e3:.1f}", f"{t / n / 1e3:.2f}", f"{mn / 1e3:.2f}", f"{mx / 1e3:.2f}",
                    f"{100 * t / total:.2f}", g])


if __name__ == "__main__":
    main()
