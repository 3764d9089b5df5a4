"""CPU-side checks of the drop-in boundary (no GPU compute).

* libmhq_huff.so loads and exports every symbol include/mhq_huff.h declares;
* the host-built code table equals the reference's (hc/huffmantable.go);
* the product package never reaches the oracle;
* without a gfx950 device the codec fails loudly instead of falling back.
"""
import ctypes
import os
import re

import pytest

from tests.conftest import REPO

HEADER = os.path.join(REPO, "include", "mhq_huff.h")


@pytest.fixture(scope="module")
def lib():
    from minhq_amd import build

    build.build()
    from minhq_amd import _lib

    return _lib.load()


def declared_symbols():
    src = open(HEADER).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    return sorted(set(re.findall(r"\b(mhq_\w+)\s*\(", src)))


def test_header_declares_entry_points():
    syms = declared_symbols()
    for s in ["mhq_open", "mhq_close", "mhq_huff_encode_len", "mhq_huff_encode", "mhq_huff_decode",
              "mhq_huff_decode_dev", "mhq_huff_encode_dev"]:
        assert s in syms


def test_library_exports_every_declared_symbol(lib):
    from minhq_amd import _lib

    for s in declared_symbols():
        assert hasattr(lib, s), s
        assert s in _lib.SIGNATURES, f"{s} has no ctypes signature"
    # and the binding declares nothing the header does not
    assert sorted(_lib.SIGNATURES) == declared_symbols()


def test_exports_are_c_symbols(lib):
    # C linkage: the dynamic symbol table carries the plain names
    import subprocess

    out = subprocess.run(["nm", "-D", "--defined-only", os.path.join(REPO, "minhq_amd", "libmhq_huff.so")],
                         capture_output=True, text=True, check=True).stdout
    names = {line.split()[-1] for line in out.splitlines() if line.strip()}
    for s in declared_symbols():
        assert s in names


def test_code_table_matches_reference(lib, golden):
    from minhq_amd.hc import code_table

    lens, code = code_table()
    ref = golden("huffman_table.json")
    assert lens == [r["len"] for r in ref]
    assert code == [r["val"] for r in ref]


def test_strerror(lib):
    assert lib.mhq_strerror(0) == b"ok"
    assert b"gfx950" in lib.mhq_strerror(-19)


def test_product_does_not_import_oracle():
    pkg = os.path.join(REPO, "minhq_amd")
    for root, _, files in os.walk(pkg):
        for f in files:
            if f.endswith((".py", ".cpp", ".hip", ".h")):
                text = open(os.path.join(root, f)).read()
                assert "import oracle" not in text and "from oracle" not in text, f
                assert not re.search(r"#include\s*[<\"].*huff_oracle", text), f
                assert "liboracle" not in text, f


def test_no_device_fails_loudly(lib):
    import torch

    if torch.cuda.is_available():
        pytest.skip("a GPU is present")
    h = ctypes.c_void_p()
    rc = lib.mhq_open(ctypes.byref(h), 0)
    assert rc == -19  # MHQ_ENODEV: no CPU fallback exists
    from minhq_amd import hc
    from minhq_amd._lib import MhqError

    with pytest.raises(MhqError):
        hc.Codec()


def test_host_helpers_pack_and_capacity():
    import numpy as np

    from minhq_amd import hc

    data, off = hc.pack([b"ab", b"", b"cde"])
    assert data.tobytes() == b"abcde" and list(off) == [0, 2, 2, 5]
    assert hc.unpack(data, off) == [b"ab", b"", b"cde"]
    cap = hc.capacity_offsets(np.array([0, 5, 5, 13], dtype=np.uint64))
    assert list(cap) == [0, 8, 8, 20]
    assert hc.HuffmanChoose(10, 9) and not hc.HuffmanChoose(10, 10)
    assert hc.HuffmanChoose(10, 12, hc.HuffmanCodingAlways)
    assert not hc.HuffmanChoose(10, 1, hc.HuffmanCodingNever)
