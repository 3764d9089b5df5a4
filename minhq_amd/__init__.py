"""minhq_amd -- MI355X-native batch codec for HPACK/QPACK Huffman string literals.

The compute path is libmhq_huff.so (hand-written gfx950 HIP kernels behind the
C ABI in include/mhq_huff.h).  `minhq_amd.hc` is the host-side mirror of the
reference's `hc` Huffman surface; `minhq_amd.workloads` builds the synthetic
batches of BASELINE.json's configs.
"""
from ._lib import LIB_PATH, MhqError, load  # noqa: F401

__all__ = ["LIB_PATH", "MhqError", "load"]
