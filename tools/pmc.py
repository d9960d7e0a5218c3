"""Summarise a rocprofv3 --pmc database: per kernel (name filter) average counter value per dispatch.

usage: python tools/pmc.py <results.db> [--match SUBSTR] [--json out.json]
FETCH_SIZE / WRITE_SIZE are reported in KB by rocprofv3; on gfx950 FETCH_SIZE counts ~1/2 of the
bytes of wide coalesced reads (MI355X_MICROARCH.md §HBM) — `corrected` doubles it.
"""
import argparse
import json
import re
import sqlite3


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("db")
    ap.add_argument("--match", default="")
    ap.add_argument("--json")
    a = ap.parse_args()
    con = sqlite3.connect(a.db)
    rows = con.execute("select kernel_name, counter_name, count(*), avg(value), avg(duration) from counters_collection "
                       "group by kernel_name, counter_name").fetchall()
    out = []
    for name, ctr, n, val, dur in rows:
        if a.match not in name:
            continue
        short = re.sub(r"\(.*\)$", "", name.replace("(anonymous namespace)::", "").replace("void ", ""))[:110]
        rec = {"kernel": short, "counter": ctr, "dispatches": n, "avg_value": val, "avg_duration_ns": dur}
        if ctr in ("FETCH_SIZE", "WRITE_SIZE"):
            rec["bytes"] = val * 1024 * (2 if ctr == "FETCH_SIZE" else 1)
            rec["note"] = "KB x1024" + (" x2 (gfx950 FETCH_SIZE half-count correction)" if ctr == "FETCH_SIZE" else "")
        out.append(rec)
        print(f"{ctr:12s} n={n:4d} avg={val:12.1f} " + (f"bytes={rec.get('bytes', 0)/1e6:9.2f} MB " if 'bytes' in rec else "") + short)
    if a.json:
        json.dump(out, open(a.json, "w"), indent=1)


if __name__ == "__main__":
    main()
