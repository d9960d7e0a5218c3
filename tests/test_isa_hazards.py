"""ISA guard (CPU): no VALU instruction of the built library reads an MFMA result fewer than 7 wait states after the MFMA,
on any control-flow path.

r06 found the cause of the long-attention wrong maxima: in the r03 ordering the compiler padded the MFMA
-> VALU read on the fall-through path of the branch over the tail mask but not on the taken path, where v_max_f32 read a
v_mfma_f32_16x16x32_f16 accumulator 1 wait state after it and saw the registers' previous contents (the K fragment's
bits: running maxima of 1e3..3e3).  tools/lab/mfma_raw_lab.hip measures the result readable from 7 wait states on gfx950.
This test runs the path-aware scan (tools/dbg/mfma_raw_paths.py) over every code object of clip-ebc_amd/lib/
libebc_hip.so, so a build whose schedule reintroduces such a read fails here instead of producing NaN rows."""
import importlib.util
import os
import shutil
import subprocess
import tempfile

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
LIB = os.path.join(REPO, "clip-ebc_amd", "lib", "libebc_hip.so")
LLVM = "/opt/rocm/lib/llvm/bin"


def _code_objects(lib, work):
    """The gfx950 code objects of the library's .hip_fatbin (one offload bundle per translation unit)."""
    fb = os.path.join(work, "fb.bin")
    # an explicit output file: without one objcopy rewrites its input in place -- here the library this very process
    # may have mapped (test_abi loads it), which crashed a later test
    subprocess.run(["objcopy", "--dump-section", f".hip_fatbin={fb}", lib, os.path.join(work, "copy.so")], check=True,
                   capture_output=True)
    data = open(fb, "rb").read()
    magic = b"__CLANG_OFFLOAD_BUNDLE__"
    starts = []
    i = data.find(magic)
    while i >= 0:
        starts.append(i)
        i = data.find(magic, i + 1)
    outs = []
    for k, s in enumerate(starts):
        e = starts[k + 1] if k + 1 < len(starts) else len(data)
        part = os.path.join(work, f"b{k}.bin")
        open(part, "wb").write(data[s:e])
        co = os.path.join(work, f"k{k}.co")
        r = subprocess.run([f"{LLVM}/clang-offload-bundler", "--unbundle", "--type=o", f"--input={part}",
                            "--targets=hipv4-amdgcn-amd-amdhsa--gfx950", f"--output={co}"], capture_output=True)
        if r.returncode == 0 and os.path.getsize(co) > 0:
            outs.append(co)
    return outs


@pytest.mark.skipif(not os.path.exists(LIB) or not os.path.exists(f"{LLVM}/llvm-objdump") or not shutil.which("objcopy"),
                    reason="needs the built library and the ROCm LLVM tools")
def test_no_mfma_result_read_within_7_wait_states():
    spec = importlib.util.spec_from_file_location("mfma_raw_paths", os.path.join(REPO, "tools", "dbg", "mfma_raw_paths.py"))
    mrp = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mrp)
    kernels, short_reads = mrp.kernels, mrp.short_reads
    work = tempfile.mkdtemp()
    try:
        cos = _code_objects(LIB, work)
        assert len(cos) >= 2, "expected one code object per translation unit"
        n_mfma, bad = 0, []
        for co in cos:
            lst = subprocess.run([f"{LLVM}/llvm-objdump", "-d", "--no-show-raw-insn", co], check=True,
                                 capture_output=True, text=True).stdout.splitlines(keepends=True)
            n_mfma += sum("v_mfma" in line for line in lst)
            for name, lines in kernels(lst):
                found, ins = short_reads(lines, below=7)
                bad += [(name, d, ins[i]["op"], ins[j]["op"]) for d, i, j in found]
        assert n_mfma > 10000, n_mfma                  # the GEMM and attention objects were scanned
        assert not bad, bad[:10]
    finally:
        shutil.rmtree(work, ignore_errors=True)
