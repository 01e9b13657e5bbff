"""Summarise a rocprofv3 kernel-trace database (rocpd SQLite) into a per-kernel CSV.

usage: python tools/prof_summary.py gpurun_out/prof/run_results.db [out.csv] [--top N] [--last-ms T]
Kernel names are shortened to the template head (argument lists dropped).  ``--last-ms T`` keeps only
dispatches that start in the final T ms of the trace (steady-state decode after ``bench.py
--profile-steps``) and also prints the GPU-busy fraction of that window.
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
    last_ms = float(sys.argv[sys.argv.index("--last-ms") + 1]) if "--last-ms" in sys.argv else None
    c = sqlite3.connect(db)
    rows_all = list(c.execute("select name, duration, grid_x, workgroup_x, start, end from kernels order by start"))
    if last_ms is not None and rows_all:
        t_end = max(r[5] for r in rows_all)
        t_lo = t_end - last_ms * 1e6
        rows_all = [r for r in rows_all if r[4] >= t_lo]
        busy, cur_s, cur_e = 0, None, None
        for r in rows_all:
            if cur_e is None or r[4] > cur_e:
                if cur_e is not None:
                    busy += cur_e - cur_s
                cur_s, cur_e = r[4], r[5]
            else:
                cur_e = max(cur_e, r[5])
        if cur_e is not None:
            busy += cur_e - cur_s
        span = t_end - rows_all[0][4] if rows_all else 1
        print(f"# window {span / 1e6:.2f} ms, {len(rows_all)} dispatches, GPU busy {100 * busy / span:.1f}%",
              file=sys.stderr)
    agg = defaultdict(lambda: [0, 0, 1 << 62, 0, ""])
    for name, dur, gx, wx, _, _ in rows_all:
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
