"""The built GPU code never writes through the scalar data cache: no scalar memory stores or atomics
and no scalar-cache write-back/discard in any kernel of the product libraries (vector stores only).
Disassembles the gfx950 code objects bundled in libdxrpt.so.  CPU-only; needs the built library and
llvm-objdump (skipped without them).  Listed in .gpurunignore: no GPU run loads it."""
import os
import re
import struct
import subprocess
import tempfile

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
LIB = os.path.join(REPO, "dxrpathtracer_amd", "lib", "libdxrpt.so")
OBJDUMP = "/opt/rocm/lib/llvm/bin/llvm-objdump"
MAGIC = b"__CLANG_OFFLOAD_BUNDLE__"
FORBIDDEN = re.compile(r"\b(s_store_\w+|s_buffer_store\w*|s_scratch_store\w*|s_atomic_\w+|s_buffer_atomic_\w+|"
                       r"s_dcache_wb\w*|s_dcache_discard\w*)\b")


def code_objects(blob: bytes):
    """gfx950 code objects of every offload bundle in the library."""
    pos = blob.find(MAGIC)
    while pos >= 0:
        n = struct.unpack_from("<Q", blob, pos + 24)[0]
        off = pos + 32
        for _ in range(n):
            o, size, tlen = struct.unpack_from("<QQQ", blob, off)
            triple = blob[off + 24:off + 24 + tlen].decode(errors="replace")
            off += 24 + tlen
            if "gfx950" in triple:
                yield triple, blob[pos + o:pos + o + size]
        pos = blob.find(MAGIC, pos + 1)


@pytest.mark.skipif(not (os.path.exists(LIB) and os.path.exists(OBJDUMP)), reason="library or llvm-objdump missing")
def test_no_scalar_cache_writes():
    blob = open(LIB, "rb").read()
    objs = list(code_objects(blob))
    assert objs, "no gfx950 code object found in libdxrpt.so"
    kernels = 0
    for triple, co in objs:
        with tempfile.NamedTemporaryFile(suffix=".co") as f:
            f.write(co)
            f.flush()
            asm = subprocess.run([OBJDUMP, "-d", "--mcpu=gfx950", f.name], capture_output=True, text=True,
                                 check=True).stdout
        kernels += asm.count(">:\n")
        bad = sorted(set(FORBIDDEN.findall(asm)))
        assert not bad, (triple, bad)
    assert kernels > 20
