"""Literal sharding across devices / ranks.

Literals are independent: a batch splits into contiguous index ranges with no
exchange step, and each shard is decoded on its own device.  Ranges are
balanced by bytes (the prefix sum over the offsets), so every device gets
about the same encoded (decode) or plaintext (encode) volume.  The C library
applies the same rule inside `mhq_open(ndev > 1)` host calls
(minhq_amd/csrc/mhq_api.cpp); this module is the multi-process form used by
bench.py ranks and by callers that drive one process per GPU.
"""
from __future__ import annotations

from typing import List, Tuple

import numpy as np


def plan_shards(off: np.ndarray, parts: int) -> List[Tuple[int, int]]:
    """Splits literals [0, n) into `parts` contiguous ranges of ~equal bytes.

    `off` is the n+1 offset array of the batch.  Returns (lo, hi) per part;
    empty ranges are allowed when there are fewer literals than parts.
    """
    if parts < 1:
        raise ValueError("parts must be >= 1")
    off = np.asarray(off, dtype=np.uint64)
    n = len(off) - 1
    if n <= 0:
        return [(0, 0)] * parts
    base, total = int(off[0]), int(off[-1] - off[0])
    cuts = [0]
    for k in range(1, parts):
        target = np.uint64(base + (total * k) // parts)
        c = int(np.searchsorted(off, target, side="left"))
        cuts.append(min(max(c, cuts[-1]), n))
    cuts.append(n)
    return [(cuts[k], cuts[k + 1]) for k in range(parts)]


def shard_view(data: np.ndarray, off: np.ndarray, lo: int, hi: int) -> Tuple[np.ndarray, np.ndarray]:
    """The bytes and rebased offsets (starting at 0) of literals [lo, hi)."""
    off = np.asarray(off, dtype=np.uint64)
    a, b = int(off[lo] - off[0]), int(off[hi] - off[0])
    return data[a:b], off[lo:hi + 1] - off[lo]


def gather_offsets(parts_off: List[np.ndarray]) -> np.ndarray:
    """Concatenates per-shard offset arrays (each starting at 0) into one."""
    out = [np.zeros(1, dtype=np.uint64)]
    base = np.uint64(0)
    for o in parts_off:
        o = np.asarray(o, dtype=np.uint64)
        out.append(o[1:] + base)
        base = base + (o[-1] if len(o) else np.uint64(0))
    return np.concatenate(out)


def max_over_ranks(pg, x: float, device: str = "cpu") -> float:
    """Max of a per-rank float over the process group (None = single process)."""
    if pg is None:
        return float(x)
    import torch

    t = torch.tensor([float(x)], dtype=torch.float64, device=device)
    pg.all_reduce(t, op=pg.ReduceOp.MAX)
    return float(t.item())


def plan_shards_device(off, parts: int):
    """plan_shards on a device tensor of offsets (int64, n+1 entries), without
    copying the offsets to the host: the same cuts, as a list of (lo, hi)."""
    import torch

    if parts < 1:
        raise ValueError("parts must be >= 1")
    n = off.numel() - 1
    if n <= 0:
        return [(0, 0)] * parts
    base, total = int(off[0].item()), int((off[-1] - off[0]).item())
    targets = torch.tensor([base + (total * k) // parts for k in range(1, parts)], dtype=torch.int64,
                           device=off.device)
    cuts = [0] + [int(c) for c in torch.searchsorted(off, targets, right=False).tolist()] + [n]
    for k in range(1, parts):
        cuts[k] = min(max(cuts[k], cuts[k - 1]), n)
    return [(cuts[k], cuts[k + 1]) for k in range(parts)]
