"""ISA guard over every gfx950 code object in ``libdfd_hip.so`` (CPU test: disassembly only).

Round 5 found the fp16 fused projection backward (``k_pwl_bwd.hip``) non-reproducible: two identical
launches differed in sum(d * silu') and sum(d * silu' * xhat) -- and in nothing else
(``profiles/r05/pwl_det_slp_r05j.txt``).  The disassembly of that build holds 32 packed-f32
instructions whose source operand is read SWAPPED (``v_pk_mul_f32 ... op_sel:[0,1] op_sel_hi:[1,0]``:
the low lane reads the register pair's high half, the high lane the low half), every one of them on
the chain of exactly those two sums; the bit-reproducible bf16 instance of the same source and the
no-SLP build hold none.  The kernel now writes that epilogue on lane-ordered pairs, which leaves the
compiler nothing to swap (``k_pwl_bwd.hip``, epilogue note).  This test keeps the whole library free
of the form: any ``v_pk_{fma,mul,add}_f32`` with ``op_sel[i] = 1`` and ``op_sel_hi[i] = 0`` fails it.
"""
import os
import re
import shutil
import struct
import subprocess
import tempfile

import pytest

from deepfake_amd import _lib

OBJDUMP = "/opt/rocm/lib/llvm/bin/llvm-objdump"
MAGIC = b"__CLANG_OFFLOAD_BUNDLE__"
_PK = re.compile(r"\bv_pk_(fma|mul|add)_f32\b")
_SEL = re.compile(r"\b(op_sel|op_sel_hi):\[([01](?:,[01])*)\]")


def swapped_sources(line: str):
    """Source indices a packed-f32 instruction reads swapped (low lane <- high register and high
    lane <- low register); [] for any other instruction."""
    if not _PK.search(line):
        return []
    sel = {"op_sel": [0, 0, 0], "op_sel_hi": [1, 1, 1]}
    for name, bits in _SEL.findall(line):
        v = [int(b) for b in bits.split(",")]
        sel[name][:len(v)] = v
    nsrc = 3 if "v_pk_fma_f32" in line else 2
    return [i for i in range(nsrc) if sel["op_sel"][i] == 1 and sel["op_sel_hi"][i] == 0]


def test_detector_recognises_the_form():
    assert swapped_sources("v_pk_mul_f32 v[158:159], v[128:129], v[120:121] op_sel:[0,1] op_sel_hi:[1,0]") == [1]
    assert swapped_sources("v_pk_fma_f32 v[94:95], v[128:129], v[120:121], v[94:95] op_sel:[0,1,0] "
                           "op_sel_hi:[1,0,1]") == [1]
    # broadcasts (both lanes read one half) and plain pairs are not swaps
    assert swapped_sources("v_pk_fma_f32 v[88:89], v[108:109], v[118:119], v[88:89] op_sel_hi:[0,1,1]") == []
    assert swapped_sources("v_pk_fma_f32 v[2:3], v[4:5], v[6:7], v[8:9] op_sel:[1,0,0]") == []
    assert swapped_sources("v_pk_mov_b32 v[2:3], v[4:5], v[6:7] op_sel:[1,0]") == []


def _code_objects(fatbin: bytes):
    """gfx950 ELF images of every offload bundle in a .hip_fatbin section."""
    pos = fatbin.find(MAGIC)
    while pos >= 0:
        n = struct.unpack_from("<Q", fatbin, pos + 24)[0]
        off = pos + 32
        for _ in range(n):
            eo, es, tl = struct.unpack_from("<QQQ", fatbin, off)
            triple = fatbin[off + 24:off + 24 + tl].decode()
            off += 24 + tl
            if "gfx950" in triple and es:
                yield fatbin[pos + eo:pos + eo + es]
        pos = fatbin.find(MAGIC, pos + 1)


@pytest.mark.skipif(not os.path.exists(OBJDUMP) or shutil.which("objcopy") is None,
                    reason="llvm-objdump / objcopy not available")
def test_library_has_no_swapped_packed_f32_operands():
    with tempfile.TemporaryDirectory() as td:
        fb = os.path.join(td, "fatbin")
        subprocess.run(["objcopy", "--dump-section", f".hip_fatbin={fb}", _lib.LIB_PATH, os.path.join(td, "x.so")],
                       check=True, capture_output=True)
        data = open(fb, "rb").read()
        bad, nobj, nkern = [], 0, 0
        for i, co in enumerate(_code_objects(data)):
            p = os.path.join(td, f"co{i}.elf")
            open(p, "wb").write(co)
            dis = subprocess.run([OBJDUMP, "-d", "--mcpu=gfx950", p], check=True, capture_output=True,
                                 text=True).stdout
            nobj += 1
            func = "?"
            for line in dis.splitlines():
                if line.endswith(">:"):
                    func = line
                    nkern += 1
                elif swapped_sources(line):
                    bad.append(f"{func} {line.strip()}")
        assert nobj >= 20 and nkern > 100, (nobj, nkern)  # every translation unit was scanned
        assert not bad, f"{len(bad)} swapped packed-f32 operand reads, e.g. {bad[:3]}"
