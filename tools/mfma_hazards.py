"""Distance (in issued instructions / wait states) from each v_mfma to the first later non-MFMA instruction that reads
or overwrites its destination registers, in straight-line order of an llvm-objdump listing of one kernel.

usage: python tools/mfma_hazards.py kernel.s [--max 20]
Each s_nop N counts N + 1 wait states, every other instruction 1.  Branches are not followed (a listing's textual
order), so a distance is exact inside a basic block and an estimate across one.  Used to check the hazard recognizer's
padding between an MFMA and the VALU that reads its result (cdna_hip_programming.md §5.7 item 2)."""
import re
import sys


def regs(tok):
    m = re.fullmatch(r"v(\d+)", tok)
    if m:
        return {int(m.group(1))}
    m = re.fullmatch(r"v\[(\d+):(\d+)\]", tok)
    if m:
        return set(range(int(m.group(1)), int(m.group(2)) + 1))
    return set()


def parse(path):
    ins = []
    for line in open(path):
        line = line.split("//")[0].strip()
        if not line or line.endswith(">:") or line.startswith("<"):
            continue
        parts = line.replace(",", " ").split()
        op, args = parts[0], parts[1:]
        ins.append((op, args))
    return ins


def main():
    path = sys.argv[1]
    mx = int(sys.argv[sys.argv.index("--max") + 1]) if "--max" in sys.argv else 20
    ins = parse(path)
    hist = {}
    worst = []
    for i, (op, args) in enumerate(ins):
        if not op.startswith("v_mfma"):
            continue
        dst = regs(args[0])
        ws = 0
        for j in range(i + 1, min(len(ins), i + 200)):
            op2, a2 = ins[j]
            if op2.startswith("s_nop"):
                ws += int(a2[0]) + 1
                continue
            if op2.startswith(("s_cbranch", "s_branch", "s_endpgm", "s_setpc")):
                break
            used = set()
            for t in a2:
                used |= regs(t)
            if op2.startswith("v_mfma"):
                # an MFMA taking the whole destination as its accumulator (src C) is the chained form
                if used & dst and regs(a2[-1]) != dst:
                    worst.append((ws, i, op, j, op2, "mfma A/B reads"))
                    break
                ws += 1
                continue
            if used & dst:
                worst.append((ws, i, op, j, op2, "reads/writes"))
                hist[ws] = hist.get(ws, 0) + 1
                break
            ws += 1
    worst.sort()
    print("first non-MFMA consumer of an MFMA result, wait states between -> count:",
          dict(sorted(hist.items())[:mx]))
    for w, i, op, j, op2, why in worst[:12]:
        print(f"  {w:3d} states: [{i}] {op} -> [{j}] {op2} ({why})")


if __name__ == "__main__" and "--war" not in sys.argv:
    main()


def war_srcab(ins, window=24):
    """(wait states, i, j, op2): a non-MFMA instruction j whose DESTINATION overlaps the A/B source registers of an
    MFMA i issued fewer than `window` wait states earlier (a VALU overwriting an in-flight MFMA's A/B operands)."""
    out = []
    for i, (op, args) in enumerate(ins):
        if not op.startswith("v_mfma"):
            continue
        srcab = regs(args[1]) | regs(args[2])
        ws = 0
        for j in range(i + 1, min(len(ins), i + 64)):
            op2, a2 = ins[j]
            if op2.startswith("s_nop"):
                ws += int(a2[0]) + 1
            else:
                if op2.startswith(("s_cbranch", "s_branch", "s_endpgm")):
                    break
                if op2.startswith(("v_", "ds_read", "global_load", "buffer_load")) and not op2.startswith("v_mfma") and a2:
                    if regs(a2[0]) & srcab:
                        out.append((ws, i, j, op2))
                        break
                ws += 1
            if ws >= window:
                break
    return out


def main_war():
    ins = parse(sys.argv[1])
    hits = war_srcab(ins)
    print(f"VALU / load writes to an MFMA's A/B source registers within 24 wait states: {len(hits)}")
    for w, i, j, op2 in sorted(hits)[:12]:
        print(f"  {w:3d} states: [{i}] {ins[i][0]} {' '.join(ins[i][1])} -> [{j}] {op2} {' '.join(ins[j][1])}")


if __name__ == "__main__" and "--war" in sys.argv:
    main_war()
