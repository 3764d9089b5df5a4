"""The shipped kernels' compiled resources (CPU only: reads libmhq_huff.so).

Round 6 (DESIGN.md "The read path's illegal memory access"):
the read kernels used to call two out-of-line helpers (the checked loop and
the streamed long literals).  Everything live across those calls spilled --
read_fused_kernel 11 VGPRs + 74 SGPRs, 48 B of scratch a lane;
read_fallback_kernel 22 VGPRs, 64 B -- and the callees reached LDS through
generic (flat) addresses.  Those are the read path's only scratch traffic,
its only flat accesses and its only cross-call register state: the memory
operations the skip-and-record guards of the faulting debug build did not
cover.  The kGaps decode now inlines both helpers; these tests pin that no
kernel of the library has scratch, spills VGPRs or uses a dynamic stack, and
that the read kernels contain no call, flat or scratch instruction.
"""
from __future__ import annotations

import os

import pytest

from tests.code_object import all_kernels, disassembly, objdump

from minhq_amd import _lib

READ_KERNELS = ("read_fused_kernel", "read_fallback_kernel", "decode_kernelILb1E")


@pytest.fixture(scope="module")
def kernels():
    if not os.path.exists(_lib.LIB_PATH):
        pytest.skip("libmhq_huff.so not built")
    return all_kernels(_lib.LIB_PATH)


def test_every_kernel_scratch_free(kernels):
    assert len(kernels) >= 20
    bad = {n: (k[".private_segment_fixed_size"], k[".vgpr_spill_count"], k[".uses_dynamic_stack"])
           for n, k in kernels.items()
           if k[".private_segment_fixed_size"] or k[".vgpr_spill_count"] or k[".uses_dynamic_stack"]}
    assert not bad, bad


def test_read_kernels_present(kernels):
    for r in READ_KERNELS:
        assert any(r in n for n in kernels), r


def test_read_kernels_no_call_flat_or_scratch():
    if not os.path.exists(_lib.LIB_PATH):
        pytest.skip("libmhq_huff.so not built")
    if objdump() is None:
        pytest.skip("llvm-objdump not found")
    funcs = disassembly(_lib.LIB_PATH)
    seen = 0
    for name, insts in funcs.items():
        if not any(r in name for r in READ_KERNELS):
            continue
        seen += 1
        bad = sorted({i for i in insts if i.startswith(("flat_", "scratch_", "s_swappc", "s_setpc"))})
        assert not bad, (name, bad)
    assert seen >= len(READ_KERNELS)
