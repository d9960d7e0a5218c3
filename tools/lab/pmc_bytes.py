"""Per-kernel-name averages of rocprofv3 --pmc counters (lab) for every kernel whose name matches a pattern: FETCH_SIZE
and WRITE_SIZE as MB (FETCH_SIZE x 1024 x 2 bytes -- gfx950 counts half of wide coalesced reads -- and WRITE_SIZE x 1024,
as tools/pmc_step.py), other counters raw.
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
SCALE = {"FETCH_SIZE": 2048 / 1e6, "WRITE_SIZE": 1024 / 1e6}
for name, cs in sorted(acc.items()):
    parts = [f"{cn}{' MB' if cn in SCALE else ''} {sum(v) / len(v) * SCALE.get(cn, 1.0):.4g}" for cn, v in sorted(cs.items())]
    print(f"{name}\n    n={len(next(iter(cs.values())))}  " + "  ".join(parts))
