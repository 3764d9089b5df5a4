"""The gfx950 code objects inside libmhq_huff.so, for tests that check the
compiled kernels' resources (no GPU needed).

The library's `.hip_fatbin` section holds one clang offload bundle per
translation unit; each bundle's `hipv4-amdgcn-amd-amdhsa--gfx950` entry is an
ELF code object whose `NT_AMDGPU_METADATA` note (msgpack) lists every
kernel's resources: `.private_segment_fixed_size` (scratch bytes a lane),
`.vgpr_spill_count`, `.sgpr_spill_count`, `.uses_dynamic_stack`.
"""
from __future__ import annotations

import os
import shutil
import struct
import subprocess
import tempfile

import msgpack

_MAGIC = b"__CLANG_OFFLOAD_BUNDLE__"
_TARGET = b"hipv4-amdgcn-amd-amdhsa--gfx950"
NT_AMDGPU_METADATA = 32


def _sections(elf: bytes):
    shoff = struct.unpack_from("<Q", elf, 0x28)[0]
    shentsize, shnum, shstrndx = struct.unpack_from("<HHH", elf, 0x3A)
    raw = [struct.unpack_from("<IIQQQQ", elf, shoff + i * shentsize) for i in range(shnum)]
    stroff = raw[shstrndx][4]

    def name(n):
        end = elf.index(b"\0", stroff + n)
        return elf[stroff + n:end].decode()

    return {name(r[0]): (r[1], r[4], r[5]) for r in raw}  # name -> (type, offset, size)


def code_objects(lib_path: str) -> list[bytes]:
    """The gfx950 ELF code objects of the library, one per translation unit."""
    data = open(lib_path, "rb").read()
    _, off, size = _sections(data)[".hip_fatbin"]
    blob = data[off:off + size]
    out = []
    start = blob.find(_MAGIC)
    while start >= 0:
        n = struct.unpack_from("<Q", blob, start + len(_MAGIC))[0]
        p = start + len(_MAGIC) + 8
        for _ in range(n):
            eoff, esize, tlen = struct.unpack_from("<QQQ", blob, p)
            triple = blob[p + 24:p + 24 + tlen]
            p += 24 + tlen
            if triple == _TARGET and esize:
                out.append(blob[start + eoff:start + eoff + esize])
        start = blob.find(_MAGIC, start + 1)
    return out


def kernel_metadata(co: bytes) -> list[dict]:
    """amdhsa.kernels of one code object (from its metadata note)."""
    for name, (typ, off, size) in _sections(co).items():
        if typ != 7:  # SHT_NOTE
            continue
        p = off
        while p < off + size:
            namesz, descsz, ntype = struct.unpack_from("<III", co, p)
            nm = co[p + 12:p + 12 + namesz]
            d0 = p + 12 + ((namesz + 3) & ~3)
            if ntype == NT_AMDGPU_METADATA and nm.rstrip(b"\0") == b"AMDGPU":
                md = msgpack.unpackb(co[d0:d0 + descsz], raw=False)
                return md["amdhsa.kernels"]
            p = d0 + ((descsz + 3) & ~3)
    return []


def all_kernels(lib_path: str) -> dict[str, dict]:
    """Every kernel of the library by mangled name."""
    ks = {}
    for co in code_objects(lib_path):
        for k in kernel_metadata(co):
            ks[k[".name"]] = k
    return ks


def objdump() -> str | None:
    for p in ("/opt/rocm/lib/llvm/bin/llvm-objdump", shutil.which("llvm-objdump") or ""):
        if p and os.path.exists(p):
            return p
    return None


def disassembly(lib_path: str) -> dict[str, list[str]]:
    """Instruction mnemonics per function symbol of every code object
    (needs llvm-objdump)."""
    tool = objdump()
    funcs: dict[str, list[str]] = {}
    with tempfile.TemporaryDirectory() as d:
        for i, co in enumerate(code_objects(lib_path)):
            path = os.path.join(d, f"co{i}.o")
            open(path, "wb").write(co)
            txt = subprocess.run([tool, "-d", "--no-show-raw-insn", path], capture_output=True, text=True,
                                 check=True).stdout
            cur = None
            for line in txt.splitlines():
                if line.endswith(">:"):
                    cur = line.split("<", 1)[1][:-2]
                    funcs[cur] = []
                elif cur and line.startswith("\t"):
                    funcs[cur].append(line.split()[0])
    return funcs
