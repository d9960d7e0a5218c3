"""Minimum wait states, over every control-flow path, from each v_mfma to the first later instruction that reads its
destination registers (llvm-objdump listing of ONE kernel, tools/isa.sh).  tools/mfma_hazards.py measures textual
distance only; this one follows s_branch / s_cbranch_* targets and fall-through, so a read reached through a taken
branch is measured on that path (r06: the r03 long-attention ordering).

usage: python tools/dbg/mfma_raw_paths.py listing.s [--below 7]   (any number of kernels)
Each s_nop N counts N + 1 wait states, every other instruction 1 (the compiler's count; tools/lab/mfma_raw_lab.hip
measures a VALU read of a v_mfma_f32_16x16x32_f16 result correct from 7 states)."""
import heapq
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


def parse(lines):
    ins = []
    for line in lines:
        code, _, cmt = line.partition("//")
        code = code.strip()
        if not code or code.endswith(">:") or code.startswith("<"):
            continue
        m = re.search(r"([0-9A-F]{8,})", cmt)
        addr = int(m.group(1), 16) if m else None
        target = None
        parts = code.replace(",", " ").split()
        op, args = parts[0], parts[1:]
        if op.startswith("s_cbranch") or op == "s_branch":
            mt = re.search(r"<[^>]*\+0x([0-9a-f]+)>", line)        # '<func+0xOFF>': offset from the function start
            target = int(mt.group(1), 16) if mt else None
        ins.append({"op": op, "args": args, "addr": addr, "toff": target})
    return ins


def short_reads(lines, below=7):
    """(wait states, mfma index, reader index, instructions) for every non-MFMA vector instruction that reads an
    MFMA's destination within < below wait states along some control-flow path of ONE kernel's listing."""
    ins = parse(lines)
    if not ins or ins[0]["addr"] is None:
        return [], ins
    base = ins[0]["addr"]
    idx_of = {x["addr"] - base: i for i, x in enumerate(ins) if x["addr"] is not None}

    def succ(i):
        x = ins[i]
        if x["op"] == "s_endpgm":
            return []
        out = []
        if x["toff"] is not None and x["toff"] in idx_of:
            out.append(idx_of[x["toff"]])
        if x["op"] != "s_branch" and i + 1 < len(ins):
            out.append(i + 1)
        return out

    def cost(i):
        x = ins[i]
        return int(x["args"][0]) + 1 if x["op"] == "s_nop" else 1

    found = []
    for i, x in enumerate(ins):
        if not x["op"].startswith("v_mfma"):
            continue
        dst = regs(x["args"][0])
        # Dijkstra over instructions: distance = wait states issued after the MFMA before instruction j
        dist = {}
        pq = [(0, j) for j in succ(i)]
        while pq:
            d, j = heapq.heappop(pq)
            if j in dist or d >= below:
                continue
            dist[j] = d
            y = ins[j]
            reads = set().union(*[regs(a) for a in y["args"][1:]]) if len(y["args"]) > 1 else set()
            writes = regs(y["args"][0]) if y["args"] else set()
            if y["op"].startswith("v_mfma"):
                if dst & writes:
                    continue                      # a later MFMA redefines it (MFMA -> MFMA chains: not a VALU read)
            elif not y["op"].startswith("s_") and (dst & reads):
                found.append((d, i, j))
                continue
            elif dst & writes and not y["op"].startswith("s_"):
                continue
            for k in succ(j):
                heapq.heappush(pq, (d + cost(j), k))
    found.sort()
    return found, ins


def kernels(listing_lines):
    """Split an llvm-objdump listing into (kernel name, lines)."""
    out, cur, buf = [], None, []
    for line in listing_lines:
        m = re.match(r"^[0-9a-f]+ <(.*)>:", line)
        if m:
            if cur is not None:
                out.append((cur, buf))
            cur, buf = m.group(1), [line]
        elif cur is not None:
            buf.append(line)
    if cur is not None:
        out.append((cur, buf))
    return out


def main():
    path = sys.argv[1]
    below = int(sys.argv[sys.argv.index("--below") + 1]) if "--below" in sys.argv else 7
    total = 0
    for name, lines in kernels(open(path)):
        found, ins = short_reads(lines, below)
        total += len(found)
        for d, i, j in found[:10]:
            print(f"  {d:2d} states: [{i}] {ins[i]['op']} {' '.join(ins[i]['args'][:2])} -> [{j}] {ins[j]['op']} "
                  f"{' '.join(ins[j]['args'][:3])}   [{name[:80]}]")
    print(f"{path}: {total} reads of an MFMA result reachable within < {below} wait states")


if __name__ == "__main__":
    main()
