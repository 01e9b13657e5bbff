"""Prefill steps in a rocprofv3 kernel trace (rocpd SQLite): per step (a run of hipBLASLt GEMMs with < 1 ms
between them), the span from its first to its last kernel, the summed kernel time, the idle time and the
largest idle gaps (where the GPU waited for the host).

usage: python tools/prefill_gaps.py DB [--min-gemms 64] [--detail] [--series SUBSTR[,SUBSTR...]]

--series: the per-launch durations (us, in launch order) of the kernels whose name contains SUBSTR -- whether a
slow kernel is slow in every layer or only at the step's start (clock ramp after idle)."""
import sqlite3
import sys


def main():
    db = sys.argv[1]
    min_g = int(sys.argv[sys.argv.index("--min-gemms") + 1]) if "--min-gemms" in sys.argv else 64
    rows = list(sqlite3.connect(db).execute("select name, start, end from kernels order by start"))
    steps, cur, last_g = [], [], None
    for i, (name, s, e) in enumerate(rows):
        if name.startswith("Cijk_"):
            if last_g is not None and s - last_g > 1e6:
                steps.append(cur)
                cur = []
            cur.append(i)
            last_g = e
    if cur:
        steps.append(cur)
    for st in steps:
        if len(st) < min_g:
            continue
        i0, i1 = st[0], st[-1]
        # extend to the step's non-GEMM kernels: back to the previous gap > 200 us, forward to the next one
        while i0 > 0 and rows[i0][1] - rows[i0 - 1][2] < 2e5:
            i0 -= 1
        while i1 + 1 < len(rows) and rows[i1 + 1][1] - rows[i1][2] < 2e5:
            i1 += 1
        win = rows[i0:i1 + 1]
        span = win[-1][2] - win[0][1]
        busy, gaps, ce = 0, [], win[0][1]
        for name, s, e in win:
            if s > ce:
                gaps.append((s - ce, name[:60]))
            busy += max(0, e - max(s, ce))
            ce = max(ce, e)
        gaps.sort(reverse=True)
        print(f"step: {len(st)} GEMMs, {len(win)} kernels, span {span / 1e6:.3f} ms, busy {busy / 1e6:.3f} ms, "
              f"idle {(span - busy) / 1e6:.3f} ms; largest gaps (us): "
              + ", ".join(f"{g / 1e3:.1f} before {n}" for g, n in gaps[:5]))
        if "--detail" in sys.argv:  # per-kernel totals of the step (us): which kernels the span is made of
            tot = {}
            for name, s, e in win:
                k = name[:70]
                n, t = tot.get(k, (0, 0.0))
                tot[k] = (n + 1, t + (e - s) / 1e3)
            for k, (n, t) in sorted(tot.items(), key=lambda kv: -kv[1][1])[:8]:
                print(f"    {t:9.1f} us  {n:4d} x {t / n:7.2f}  {k}")
        if "--series" in sys.argv:
            for sub in sys.argv[sys.argv.index("--series") + 1].split(","):
                ds = [(e - s) / 1e3 for name, s, e in win if sub in name]
                if ds:
                    print(f"    series {sub}: " + " ".join(f"{d:.1f}" for d in ds))


if __name__ == "__main__":
    main()
