"""In-tree build of libmhq_huff.so for gfx950 (hipcc, no JIT cache).

The shared library is written next to this file so that it travels with the
repository snapshot to the GPU box (it is git-ignored, not gpurun-ignored).
"""
from __future__ import annotations

import os
import subprocess
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
CSRC = os.path.join(HERE, "csrc")
LIB = os.path.join(HERE, "libmhq_huff.so")
SOURCES = ["huff_decode.hip", "huff_decode_stream.hip", "read_strings.hip", "huff_encode.hip", "enc_packed.hip", "huff_scan.hip", "str_frame.hip", "huff_table.cpp", "mhq_api.cpp"]
HEADERS = ["huff_kernels.h", "huff_decode_dev.h", "huff_encode_dev.h", "huff_common.h", "huff_table.h", os.path.join("..", "..", "include", "mhq_huff.h")]
ARCH = os.environ.get("MHQ_OFFLOAD_ARCH", "gfx950")


def _hipcc() -> str:
    for cand in (os.environ.get("HIPCC"), "/opt/rocm/bin/hipcc", "hipcc"):
        if cand and (os.path.sep not in cand or os.path.exists(cand)):
            return cand
    raise RuntimeError("hipcc not found")


def _stale() -> bool:
    if not os.path.exists(LIB):
        return True
    t = os.path.getmtime(LIB)
    deps = [os.path.join(CSRC, f) for f in SOURCES + HEADERS]
    return any(os.path.getmtime(p) > t for p in deps if os.path.exists(p))


def build(force: bool = False, verbose: bool = False) -> str:
    if not force and not _stale():
        return LIB
    cmd = [_hipcc(), f"--offload-arch={ARCH}", "-O3", "-std=c++17", "-fPIC", "-shared", "-Wall",
           "-o", LIB + ".tmp"] + [os.path.join(CSRC, f) for f in SOURCES]
    if verbose:
        print(" ".join(cmd), file=sys.stderr)
    subprocess.check_call(cmd)
    os.replace(LIB + ".tmp", LIB)
    return LIB


if __name__ == "__main__":
    print(build(force="--force" in sys.argv, verbose=True))
