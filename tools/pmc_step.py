"""In-step PMC per kernel class: rocprofv3 --pmc passes over the bench command itself, cut to its timed steps.

usage: python tools/pmc_step.py --classes classes.json DIR [DIR ...] [--json out.json]

Each DIR holds one `rocprofv3 --pmc <counters> -- python3 bench.py ... --classes-out classes.json` database.  The
dispatches between the two `ebc_marker_kernel` launches (bench.py's timed steps) are split by kernel family
(gemm_nt_kernel, attn_*, ln_*, dace_loss_kernel, as bench.py's probe kinds); within a family the k-th dispatch is
launch k mod (the family's launches per step) of the step, whose class (shape + epilogue) `classes.json` lists in
launch order.  Per class: the mean of every counter and of the dispatch duration, then
  fetch_bytes  = FETCH_SIZE x 1024 x 2   (gfx950 FETCH_SIZE counts half of wide coalesced reads, MI355X_MICROARCH.md §HBM)
  write_bytes  = WRITE_SIZE x 1024
  traffic      = fetch_bytes + write_bytes          (L2 <-> fabric bytes per launch: MALL hits included)
  mfma_busy    = SQ_VALU_MFMA_BUSY_CYCLES / (duration x 2.4 GHz x 1024 SIMDs): the fraction of the launch's SIMD
                 cycles the matrix pipes were busy, at the 2.4 GHz maximum clock (the chip runs at or below it, so
                 this is a lower bound; SQ_VALU_MFMA_BUSY_CYCLES counts 16 per v_mfma_f32_16x16x32_f16)
  mfma_busy_sq = SQ_VALU_MFMA_BUSY_CYCLES / (SQ_BUSY_CYCLES / 32 x 1024): the same over the cycles the shader
                 engines held waves (32 SEs; also low for a launch that leaves CUs idle)
  sq_clock_ghz = SQ_BUSY_CYCLES / 32 / duration (<= 2.4; r03's GRBM_GUI_ACTIVE / 8 read up to 6.9 GHz on launches
                 shorter than the counter window, so it is no longer used)
  valu_per_mfma= SQ_INSTS_VALU / SQ_INSTS_MFMA (third pass)
  l2_hit       = TCC_HIT_sum / (TCC_HIT_sum + TCC_MISS_sum)
"""
import argparse
import glob
import json
import os
import sqlite3
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from bench import family_of  # noqa: E402


def dispatches(db):
    con = sqlite3.connect(db)
    rows = con.execute("select dispatch_id, kernel_name, counter_name, value, start, end from counters_collection").fetchall()
    out = {}
    for did, name, ctr, val, st, en in rows:
        d = out.setdefault(did, {"name": name, "start": st, "end": en, "c": {}})
        d["c"][ctr] = d["c"].get(ctr, 0.0) + val
    return [out[k] for k in sorted(out)]


def classify(disp, order):
    marks = [i for i, d in enumerate(disp) if "ebc_marker_kernel" in d["name"]]
    if len(marks) < 2:
        raise SystemExit(f"{len(marks)} ebc_marker_kernel dispatches (need the two around the timed steps)")
    win = disp[marks[0] + 1:marks[1]]
    per_fam = {}
    for o in order:
        per_fam.setdefault(o["family"], []).append(o["kernel"])
    seen = {}
    out = []
    for d in win:
        fam = family_of(d["name"])
        if fam is None or fam not in per_fam:
            continue
        k = seen.get(fam, 0)
        seen[fam] = k + 1
        out.append((per_fam[fam][k % len(per_fam[fam])], d))
    for fam, n in seen.items():
        if n % len(per_fam[fam]):
            raise SystemExit(f"family {fam}: {n} dispatches in the window, not a multiple of {len(per_fam[fam])} per step")
    return out, {fam: n // len(per_fam[fam]) for fam, n in seen.items()}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--classes", required=True)
    ap.add_argument("dirs", nargs="+")
    ap.add_argument("--json")
    a = ap.parse_args()
    order = json.load(open(a.classes))["launches"]
    agg = {}
    steps = None
    for d in a.dirs:
        for db in glob.glob(os.path.join(d, "**", "*.db"), recursive=True):
            pairs, st = classify(dispatches(db), order)
            steps = st
            for key, disp in pairs:
                c = agg.setdefault(key, {"kernel": key, "n": {}, "sum": {}, "dur_sum": 0.0, "dur_n": 0})
                for ctr, v in disp["c"].items():
                    c["sum"][ctr] = c["sum"].get(ctr, 0.0) + v
                    c["n"][ctr] = c["n"].get(ctr, 0) + 1
                c["dur_sum"] += disp["end"] - disp["start"]
                c["dur_n"] += 1
    out = []
    for c in agg.values():
        m = {k: c["sum"][k] / c["n"][k] for k in c["sum"]}
        r = {"kernel": c["kernel"], "dispatches": c["dur_n"], "avg_duration_us": round(c["dur_sum"] / c["dur_n"] / 1e3, 3),
             "counters": m}
        if "FETCH_SIZE" in m:
            r["fetch_bytes"] = m["FETCH_SIZE"] * 1024 * 2
        if "WRITE_SIZE" in m:
            r["write_bytes"] = m["WRITE_SIZE"] * 1024
        if "fetch_bytes" in r and "write_bytes" in r:
            r["traffic_bytes_per_launch"] = r["fetch_bytes"] + r["write_bytes"]
        dur_ns = c["dur_sum"] / c["dur_n"] if c["dur_n"] else 0.0
        if "SQ_VALU_MFMA_BUSY_CYCLES" in m and dur_ns:
            r["mfma_busy_frac"] = m["SQ_VALU_MFMA_BUSY_CYCLES"] / (dur_ns * 1e-9 * 2.4e9 * 1024)
        if m.get("SQ_BUSY_CYCLES") and dur_ns:
            r["sq_clock_ghz"] = m["SQ_BUSY_CYCLES"] / 32 / dur_ns
            if "SQ_VALU_MFMA_BUSY_CYCLES" in m:
                r["mfma_busy_sq"] = m["SQ_VALU_MFMA_BUSY_CYCLES"] / (m["SQ_BUSY_CYCLES"] / 32 * 1024)
        if m.get("SQ_INSTS_MFMA"):
            r["valu_per_mfma"] = m.get("SQ_INSTS_VALU", 0.0) / m["SQ_INSTS_MFMA"]
        if m.get("TCC_HIT_sum") is not None and m.get("TCC_MISS_sum") is not None:
            r["l2_hit"] = m["TCC_HIT_sum"] / max(1.0, m["TCC_HIT_sum"] + m["TCC_MISS_sum"])
        out.append(r)
    out.sort(key=lambda r: -r["avg_duration_us"] * r["dispatches"])
    for r in out:
        print(json.dumps({k: (round(v, 4) if isinstance(v, float) else v) for k, v in r.items() if k != "counters"}))
    if a.json:
        json.dump({"steps_per_family": steps, "classes": out}, open(a.json, "w"), indent=1)


if __name__ == "__main__":
    main()
