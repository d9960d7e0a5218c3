"""Per-kernel-name averages of rocprofv3 --pmc counters (lab): FETCH_SIZE / WRITE_SIZE (KB, gfx950 TCC units as the
bench's pmc_step.py reads them) for every kernel whose name matches a pattern.
    python tools/lab/pmc_bytes.py DB [DB ...] --match prep_weights transpose im2col"""
import argparse
import collections
import sqlite3

ap = argparse.ArgumentParser()
ap.add_argument("dbs", nargs="+")
ap.add_argument("--match", nargs="+", default=[""])
a = ap.parse_args()
acc = collections.defaultdict(lambda: collections.defaultdict(list))
dur = collections.defaultdict(list)
for db in a.dbs:
    con = sqlite3.connect(db)
    per = collections.defaultdict(dict)
    for did, name, cn, v, s, e in con.execute("select dispatch_id, kernel_name, counter_name, value, start, end "
                                              "from counters_collection"):
        if any(m in name for m in a.match):
            per[(did, name)][cn] = per[(did, name)].get(cn, 0.0) + v
            per[(did, name)]["_dur"] = (e - s) / 1000.0
    for (did, name), cs in per.items():
        for cn, v in cs.items():
            acc[name[:90]][cn].append(v)
for name, cs in sorted(acc.items()):
    parts = [f"{cn} {sum(v) / len(v):.4g}" for cn, v in sorted(cs.items())]
    print(f"{name}\n    n={len(next(iter(cs.values())))}  " + "  ".join(parts))
