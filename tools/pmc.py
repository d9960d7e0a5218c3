"""Summarise rocprofv3 --pmc databases: per kernel, the average counter value per dispatch.

usage: python tools/pmc.py <results.db> [--match SUBSTR] [--json out.json]
       python tools/pmc.py --merge DIR [DIR ...] --label TEXT --json out.json   (one pass per DIR, merged)
FETCH_SIZE / WRITE_SIZE are in KB; on gfx950 FETCH_SIZE counts ~1/2 of the bytes of wide coalesced reads
(MI355X_MICROARCH.md §HBM): `bytes` doubles it.  SQ_* cycle counters count quad-cycles except
SQ_VALU_MFMA_BUSY_CYCLES (cycles); derived: mfma_busy = MFMA busy / (GRBM_GUI_ACTIVE/8 x CUs x 4 SIMDs) when
both are present, lds_conflict = SQ_LDS_BANK_CONFLICT / SQ_LDS_IDX_ACTIVE.
"""
import argparse
import glob
import json
import os
import re
import sqlite3


def rows(db, match=""):
    con = sqlite3.connect(db)
    out = con.execute("select kernel_name, counter_name, count(*), avg(value), avg(duration) from counters_collection "
                      "group by kernel_name, counter_name").fetchall()
    for name, ctr, n, val, dur in out:
        if match and match not in name:
            continue
        short = re.sub(r"\(.*\)$", "", name.replace("(anonymous namespace)::", "").replace("void ", ""))[:110]
        yield short, ctr, n, val, dur


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("db", nargs="?")
    ap.add_argument("--match", default="")
    ap.add_argument("--json")
    ap.add_argument("--merge", nargs="*")
    ap.add_argument("--label", default="")
    a = ap.parse_args()
    if a.merge:
        kern = {}
        for d in a.merge:
            for db in glob.glob(os.path.join(d, "**", "*.db"), recursive=True):
                for short, ctr, n, val, dur in rows(db, a.match):
                    if short.startswith(("at::", "__amd", "void at::")) or "elementwise" in short or "distribution" in short:
                        continue                     # torch's operand initialisation kernels
                    k = kern.setdefault(short, {"kernel": short, "label": a.label, "dispatches": n, "counters": {}})
                    k["counters"][ctr] = val
                    k.setdefault("avg_duration_ns", dur)
        for k in kern.values():
            c = k["counters"]
            if "FETCH_SIZE" in c:
                c["fetch_bytes"] = c["FETCH_SIZE"] * 1024 * 2
            if "WRITE_SIZE" in c:
                c["write_bytes"] = c["WRITE_SIZE"] * 1024
            if "fetch_bytes" in c and "write_bytes" in c:
                k["traffic_bytes_per_launch"] = c["fetch_bytes"] + c["write_bytes"]
            if c.get("SQ_LDS_IDX_ACTIVE"):
                k["lds_conflict_frac"] = c.get("SQ_LDS_BANK_CONFLICT", 0) / c["SQ_LDS_IDX_ACTIVE"]
            if c.get("GRBM_GUI_ACTIVE") and "SQ_VALU_MFMA_BUSY_CYCLES" in c:
                k["mfma_busy_frac"] = c["SQ_VALU_MFMA_BUSY_CYCLES"] / (c["GRBM_GUI_ACTIVE"] / 8 * 256 * 4)
            if c.get("SQ_WAVE_CYCLES"):
                k["wait_any_frac"] = c.get("SQ_WAIT_ANY", 0) / c["SQ_WAVE_CYCLES"]
                k["wait_inst_any_frac"] = c.get("SQ_WAIT_INST_ANY", 0) / c["SQ_WAVE_CYCLES"]
                k["active_inst_frac"] = c.get("SQ_ACTIVE_INST_ANY", 0) / c["SQ_WAVE_CYCLES"]
                k["wait_inst_lds_frac"] = c.get("SQ_WAIT_INST_LDS", 0) / c["SQ_WAVE_CYCLES"]
            if c.get("TCC_HIT_sum") is not None and c.get("TCC_MISS_sum") is not None:
                k["l2_hit"] = c["TCC_HIT_sum"] / max(1.0, c["TCC_HIT_sum"] + c["TCC_MISS_sum"])
            if c.get("TCP_TCC_READ_REQ_sum"):
                k["l2_read_latency_cycles"] = c.get("TCP_TCC_READ_REQ_LATENCY_sum", 0) / c["TCP_TCC_READ_REQ_sum"]
        out = sorted(kern.values(), key=lambda k: -k.get("avg_duration_ns", 0))
        for k in out:
            brief = {x: (round(v, 4) if isinstance(v, float) else v) for x, v in k.items() if x not in ("counters",)}
            print(json.dumps(brief))
        if a.json:
            json.dump(out, open(a.json, "w"), indent=1)
        return
    out = []
    for short, ctr, n, val, dur in rows(a.db, a.match):
        rec = {"kernel": short, "counter": ctr, "dispatches": n, "avg_value": val, "avg_duration_ns": dur}
        if ctr in ("FETCH_SIZE", "WRITE_SIZE"):
            rec["bytes"] = val * 1024 * (2 if ctr == "FETCH_SIZE" else 1)
        out.append(rec)
        print(f"{ctr:12s} n={n:4d} avg={val:12.1f} " + (f"bytes={rec.get('bytes', 0)/1e6:9.2f} MB " if 'bytes' in rec else "") + short)
    if a.json:
        json.dump(out, open(a.json, "w"), indent=1)


if __name__ == "__main__":
    main()
