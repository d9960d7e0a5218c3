"""CPU unit test of the path-aware MFMA read scan (tools/dbg/mfma_raw_paths.py) that tests/test_isa_hazards.py runs over
the built library: on a synthetic listing shaped like the r03 long-attention failure -- an MFMA, then a
branch over the padded tail-mask block -- the read reached through the TAKEN branch one wait state after the MFMA is
reported, the padded fall-through reads are not, and a listing padded on both paths is clean."""
import importlib.util
import os

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
_spec = importlib.util.spec_from_file_location("mfma_raw_paths", os.path.join(REPO, "tools", "dbg", "mfma_raw_paths.py"))
mrp = importlib.util.module_from_spec(_spec)
_spec.loader.exec_module(mrp)


def _listing(taken_pad):
    """k: MFMA -> v[46:49]; s_cbranch_scc1 to the v46 read; fall-through: 16 wait states of s_nop, then reads of v47
    and v46.  taken_pad inserts s_nop 7 x 2 at the branch target as well."""
    body = [
        ("v_mfma_f32_16x16x32_f16 v[46:49], v[44:47], v[22:25], 0", 8),
        ("s_cbranch_scc1 3", 4),
        ("s_nop 7", 4),
        ("s_nop 7", 4),
        ("v_max_f32_e32 v42, v47, v47", 4),
    ]
    if taken_pad:
        body += [("s_nop 7", 4), ("s_nop 7", 4)]
    body += [("v_max_f32_e32 v43, v46, v46", 4), ("s_endpgm", 4)]
    addr, lines, offs = 0x1000, ["0000000000001000 <k>:\n"], []
    for op, size in body:
        offs.append(addr - 0x1000)
        lines.append([op, addr])
        addr += size
    target = offs[5]                        # the first instruction after the fall-through read of v47
    out = lines[:1]
    for op, a in lines[1:]:
        tail = f" <k+0x{target:x}>" if op.startswith("s_cbranch") else ""
        out.append(f"\t{op:58s} // {a:012X}: 00000000{tail}\n")
    return out


def test_taken_branch_read_one_state_after_mfma_is_found():
    [(name, lines)] = mrp.kernels(_listing(taken_pad=False))
    found, ins = mrp.short_reads(lines, below=7)
    assert name == "k"
    assert [(d, ins[j]["op"], ins[j]["args"][1]) for d, i, j in found] == [(1, "v_max_f32_e32", "v46")]


def test_padded_paths_are_clean():
    [(_, lines)] = mrp.kernels(_listing(taken_pad=True))
    found, _ = mrp.short_reads(lines, below=7)
    assert found == []
