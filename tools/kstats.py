"""Summarise a rocprofv3 rocpd database (``--kernel-trace`` output) as per-kernel stats.

usage: python tools/kstats.py <results.db> [--csv out.csv] [--top N] [--per STEPS] [--window] [--calls PATTERN]

Prints calls / total / average / share per kernel name (templated names shortened), and with
``--per`` the per-step time of each kernel (total / STEPS).  ``--window`` keeps only the kernels that run
between the first two `ebc_marker_kernel` launches (bench.py brackets its timed steps with them), so
warm-up, the probe pass and the CPU-baseline leg are excluded.
"""
import argparse
import csv
import re
import sqlite3


def short(name):
    name = re.sub(r"\(anonymous namespace\)::", "", name)
    name = re.sub(r"void ", "", name)
    name = re.sub(r"\(.*\)$", "", name)          # drop the argument list
    return name[:140]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("db")
    ap.add_argument("--csv")
    ap.add_argument("--top", type=int, default=40)
    ap.add_argument("--per", type=float, default=0.0)
    ap.add_argument("--window", action="store_true")
    ap.add_argument("--calls", default="", help="also list every launch whose name contains PATTERN (in time order, "
                    "with its duration and the kernel that ran before it)")
    a = ap.parse_args()
    con = sqlite3.connect(a.db)
    where = ""
    if a.window:
        cols = {r[1] for r in con.execute("pragma table_info(kernels)")}
        if not {"start", "end"} <= cols:
            raise SystemExit(f"kernels view has no start/end columns ({sorted(cols)})")
        marks = con.execute("select start, end from kernels where name like '%ebc_marker_kernel%' order by start").fetchall()
        if len(marks) < 2:
            raise SystemExit(f"--window: {len(marks)} ebc_marker_kernel launches in the trace (need 2)")
        where = f" where start > {marks[0][1]} and end < {marks[1][0]}"
        print(f"window: {(marks[1][0] - marks[0][1]) / 1e6:.3f} ms between the markers")
    rows = con.execute("select name, count(*), sum(duration), avg(duration), min(duration), max(duration) "
                       f"from kernels{where} group by name order by sum(duration) desc").fetchall()
    total = sum(r[2] for r in rows)
    out = []
    for name, n, tot, avg, mn, mx in rows:
        out.append({"kernel": short(name), "calls": n, "total_us": tot / 1e3, "avg_us": avg / 1e3,
                    "min_us": mn / 1e3, "max_us": mx / 1e3, "pct": 100.0 * tot / total,
                    "per_step_us": (tot / 1e3 / a.per) if a.per else ""})
    print(f"{'pct':>6} {'calls':>6} {'avg_us':>9} {'per_step':>9}  kernel")
    for r in out[:a.top]:
        ps = f"{r['per_step_us']:9.1f}" if a.per else ""
        print(f"{r['pct']:6.2f} {r['calls']:6d} {r['avg_us']:9.2f} {ps:>9}  {r['kernel']}")
    print(f"total kernel time {total / 1e6:.3f} ms" + (f"  per step {total / 1e3 / a.per:.1f} us" if a.per else ""))
    if a.calls:
        seq = con.execute(f"select name, start, end, duration from kernels{where} order by start").fetchall()
        t0 = seq[0][1] if seq else 0
        print(f"\n== launches matching {a.calls!r}: start_us dur_us gap_us  previous kernel")
        for i, (name, s0, e0, d) in enumerate(seq):
            if a.calls in name:
                prev = seq[i - 1] if i else None
                gap = (s0 - prev[2]) / 1e3 if prev else 0.0
                print(f"{(s0 - t0) / 1e3:10.1f} {d / 1e3:8.2f} {gap:7.2f}  {short(prev[0]) if prev else '-'}")
    if a.csv:
        with open(a.csv, "w", newline="") as f:
            w = csv.DictWriter(f, fieldnames=list(out[0].keys()))
            w.writeheader()
            w.writerows(out)


if __name__ == "__main__":
    main()
