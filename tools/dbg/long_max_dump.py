"""Long-attention wrong-maxima lab (r06): run the chunked forward (attn_fwd_long_kernel) at the
failing shape of tests/test_gpu_kernels.py::test_attention_fwd_bwd[2-257-f16] on the library EBC_LIB_PATH names and,
when that build has the EBC_LONG_MAX_DUMP hook (ebc_lab_set_lmdbg), print the per-lane chunk maxima of the rows that
come out non-finite: the lane's own tile maximum, its masked tile values, the row maximum after the cross-lane
shuffles and the running maximum -- next to the same rows of a passing build when LIB_GOOD names one.
    EBC_LIB_PATH=clip-ebc_amd/lib/lmbadd/libebc_hip.so LIB_GOOD=clip-ebc_amd/lib/lmgoodd/libebc_hip.so \
        python tools/dbg/long_max_dump.py
"""
import ctypes
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(REPO, "clip-ebc_amd"))
import numpy as np  # noqa: E402
import torch  # noqa: E402

B, L, H, LNW = 2, 257, 12, 8


def run(path):
    lib = ctypes.CDLL(path)
    dt = torch.float16
    g = torch.Generator(device="cuda").manual_seed(B * 1000 + L)
    qkv = (torch.randn(B * L, 3 * H * 64, device="cuda", generator=g) * 1.5).to(dt)
    out = torch.empty(B * L, H * 64, device="cuda", dtype=dt)
    lse = torch.empty(B, H, L, device="cuda")
    nqb = (L + 16 * LNW - 1) // (16 * LNW)
    grid = B * H * nqb
    dbg = torch.full((grid * LNW * 2 * 64 * 8,), float("nan"), device="cuda")
    has = hasattr(lib, "ebc_lab_set_lmdbg")
    if has:
        lib.ebc_lab_set_lmdbg.argtypes = [ctypes.c_void_p]
        assert lib.ebc_lab_set_lmdbg(ctypes.c_void_p(dbg.data_ptr())) == 0
    f = lib.ebc_attention_fwd
    f.argtypes = [ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int, ctypes.c_int, ctypes.c_int,
                  ctypes.c_void_p]
    EBC_F16 = 1
    rc = f(EBC_F16, qkv.data_ptr(), out.data_ptr(), lse.data_ptr(), B, L, H, ctypes.c_void_p(torch.cuda.current_stream().cuda_stream))
    assert rc == 0, rc
    torch.cuda.synchronize()
    o = out.float().view(B, L, H, 64)
    bad = (~torch.isfinite(o)).any(-1) | (~torch.isfinite(lse.permute(0, 2, 1)))     # [B, L, H]
    return bad.cpu(), dbg.view(grid, LNW, 2, 64, 8).cpu().numpy(), has, grid, nqb


def xcd_inverse(nwg):
    """blockIdx -> the (crop, head, query block) unit the kernel gives it (mfma.h xcd_remap)."""
    inv = {}
    for orig in range(nwg):
        if nwg <= 8:
            inv[orig] = orig
            continue
        q, r, x = nwg // 8, nwg % 8, orig % 8
        inv[orig] = (x * (q + 1) if x < r else r * (q + 1) + (x - r) * q) + orig // 8
    return {v: k for k, v in inv.items()}          # unit -> blockIdx


def main():
    bad, dbg, has, grid, nqb = run(os.environ["EBC_LIB_PATH"])
    rows = bad.nonzero().tolist()
    print(f"{os.environ['EBC_LIB_PATH']}: {len(rows)} non-finite (crop, query, head) rows of {B * L * H}")
    good = None
    if os.environ.get("LIB_GOOD"):
        gb, good, _, _, _ = run(os.environ["LIB_GOOD"])
        print(f"{os.environ['LIB_GOOD']}: {int(gb.sum())} non-finite rows")
    if not has:
        return
    unit2blk = xcd_inverse(grid)
    for (b, q, h) in rows[:6]:
        qb, w, fr = q // (16 * LNW), (q % (16 * LNW)) // 16, q % 16
        blk = unit2blk[(b * H + h) * nqb + qb]
        if os.environ.get("LM_END"):
            # end-of-kernel dump (EBC_LONG_MAX_DUMP placed after the chunk loop): running max m, sum, O fragments
            for fg in range(4):
                lane = fg * 16 + fr
                r = dbg[blk, w, 0, lane]
                print(f"crop {b} query {q} head {h} lane {lane:2d}: m {r[0]: .6g} sum {r[1]: .6g} o {r[2]: .4g} {r[3]: .4g} "
                      f"{r[4]: .4g} chunks {r[5]:.0f} qme {r[7]:.0f}")
            continue
        for ch in range(2):
            for fg in range(4):
                lane = fg * 16 + fr
                r = dbg[blk, w, ch, lane]
                line = (f"crop {b} query {q} head {h} chunk {ch} lane {lane:2d} (fg {fg}): lane max {r[0]: .6g}  "
                        f"tile {r[1]: .4g} {r[2]: .4g} {r[3]: .4g} {r[4]: .4g}  row max {r[5]: .6g}  running {r[6]: .6g}  nkt {r[7]:.0f}")
                if good is not None:
                    rg = good[blk, w, ch, lane]
                    line += f"   | good: lane max {rg[0]: .6g} row max {rg[5]: .6g} tile {rg[1]: .4g} {rg[2]: .4g} {rg[3]: .4g} {rg[4]: .4g}"
                print(line)


if __name__ == "__main__":
    main()
