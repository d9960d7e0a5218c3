"""Per kernel class in a rocprofv3 kernel trace of bench.py (lab): the first launch of each step vs the class mean, over
the timed steps (the window between the ebc markers), to see which launches pay for cold operands.
    python tools/lab/first_launch_stats.py gpurun_out/<dir>/run_results.db [more.db ...]"""
import collections
import re
import sqlite3
import sys


def short(n):
    n = n.replace("_ZN12_GLOBAL__N_1", "").replace("void (anonymous namespace)::", "")
    return n[:64]


def stats(db):
    con = sqlite3.connect(db)
    marks = con.execute("select start, end from kernels where name like '%ebc_marker_kernel%' order by start").fetchall()
    seq = con.execute("select name, duration from kernels where start > ? and end < ? order by start",
                      (marks[0][1], marks[-1][0])).fetchall()
    steps, cur = [], []
    for name, d in seq:
        cur.append((name, d / 1000.0))
        if "adam_kernel" in name:
            steps.append(cur)
            cur = []
    per = collections.defaultdict(lambda: [[], []])      # class -> [first launches], [other launches]
    for st in steps:
        seen = set()
        for name, d in st:
            k = short(name)
            per[k][0 if k not in seen else 1].append(d)
            seen.add(k)
    return len(steps), per


for db in sys.argv[1:]:
    n, per = stats(db)
    print(f"== {db}: {n} steps")
    for k, (first, rest) in sorted(per.items(), key=lambda kv: -sum(kv[1][0]) - sum(kv[1][1])):
        if len(rest) >= n * 5:
            f, r = sum(first) / len(first), sum(rest) / len(rest)
            print(f"  {k:64s} first {f:7.2f} us  others {r:7.2f} us  (+{f - r:5.2f})")
