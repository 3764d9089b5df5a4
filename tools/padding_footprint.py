#!/usr/bin/env python3
"""How much of a decode's capacity layout (regions of floor(8C/5) bytes) is
padding that no store granule could skip: for each granule size, the bytes in
granules that hold at least one decoded byte.  Host-only (oracle encode_len).

  python tools/padding_footprint.py
"""
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from minhq_amd import workloads  # noqa: E402
from oracle import oracle  # noqa: E402


def covered(starts, ends, total, g):
    m = np.zeros(total // g + 2, dtype=np.int64)
    np.add.at(m, starts // g, 1)
    np.add.at(m, (ends - 1) // g + 1, -1)
    return int((np.cumsum(m)[:(total + g - 1) // g] > 0).sum()) * g


def main():
    for name, lo, hi in (("northstar", 8, 56), ("config2", 8, 64)):
        b = workloads.make_batch(1 << 20, "uniform", "hdr", workloads.SEED_NORTH_STAR, lo, hi)
        el = oracle.encode_len_batch(b.data, b.off, nthreads=8).astype(np.int64)
        L = np.diff(b.off.astype(np.int64))
        co = np.concatenate([[0], np.cumsum(el * 8 // 5)])
        nz = L > 0
        s, e = co[:-1][nz], co[:-1][nz] + L[nz]
        tot = int(co[-1])
        row = {"batch": name, "decoded": int(L.sum()), "layout": tot}
        for g in (16, 32, 64):
            row[f"granules_{g}B"] = covered(s, e, tot, g)
        print(row)


if __name__ == "__main__":
    main()
