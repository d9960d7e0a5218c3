"""List the MFMA instructions of a disassembly (tools/isa.sh output) whose destination overlaps a source operand, per
kernel: full overlap (dst == src, the register allocator's usual reuse) and PARTIAL overlap (a register tuple shifted
against the source), which the r03 long-attention failure build holds (tools/lab/mfma_overlap_lab.hip).
    bash tools/isa.sh clip-ebc_amd/build/attention.o /tmp/a.s && python tools/dbg/mfma_overlap_scan.py /tmp/a.s
"""
import re
import sys


def tuple_regs(t):
    m = re.match(r"[va]\[(\d+):(\d+)\]", t)
    return set(range(int(m.group(1)), int(m.group(2)) + 1)) if m else set()


def scan(path):
    kern, rows = None, {}
    for line in open(path):
        mk = re.match(r"^[0-9a-f]+ <(.*)>:", line)
        if mk:
            kern = mk.group(1)
            continue
        m = re.search(r"v_mfma_\S+\s+([va]\[\d+:\d+\]),\s*([va]\[\d+:\d+\]),\s*([va]\[\d+:\d+\]),\s*(\S+)", line)
        if not m:
            continue
        d, a, b, c = (tuple_regs(x) for x in m.groups())
        r = rows.setdefault(kern, {"mfma": 0, "full": 0, "partial": []})
        r["mfma"] += 1
        for s, name in ((a, "A"), (b, "B"), (c, "C")):
            if d & s:
                if d == s:
                    r["full"] += 1
                else:
                    r["partial"].append((name, line.split("//")[0].strip()))
    return rows


if __name__ == "__main__":
    for path in sys.argv[1:]:
        rows = scan(path)
        tot_p = sum(len(r["partial"]) for r in rows.values())
        print(f"{path}: {sum(r['mfma'] for r in rows.values())} MFMAs, {sum(r['full'] for r in rows.values())} full and "
              f"{tot_p} partial destination/source overlaps")
        for k, r in rows.items():
            for name, ins in r["partial"]:
                print(f"  partial {name}: {ins}   [{k[:90]}]")
