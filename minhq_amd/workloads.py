"""Synthetic literal batches for BASELINE.json's configs.

Deterministic and language-neutral: splitmix64 streams, one for literal
lengths (seed) and one for literal bytes (seed ^ 0xB7E151628AED2A6A).

Byte distributions:
  hdr   -- byte frequencies of the netbsd.qif header set (errors.log:7-241,
           217 fields / 5,736 bytes / 61 distinct bytes), add-one smoothed over
           0x20..0x7E; ~5.8 bits per byte under the RFC 7541 code.
  print -- uniform over 0x20..0x7E (7.81 bits per byte).
  adv   -- uniform over the 66 bytes whose code is >= 26 bits (27.35 bits/byte).
Length distributions:
  uniform(a, b) -- U{a..b};  zipf -- P(L=k) proportional to 1/(k-3), k in 4..256.
"""
from __future__ import annotations

from dataclasses import dataclass
from typing import Tuple

import numpy as np

# netbsd.qif byte counts for 0x20..0x7E (errors.log:7-241; recomputed from
# tests/golden/netbsd_qif.json by tests/test_oracle.py::test_netbsd_histogram).
NETBSD_HIST = [
    163, 0, 0, 0, 0, 0, 0, 0, 18, 18, 36, 1, 41, 162, 181, 165, 183, 74, 19, 0, 36, 72, 36, 0, 37, 1,
    107, 75, 0, 22, 0, 0, 0, 0, 2, 1, 1, 18, 19, 36, 0, 0, 0, 0, 0, 19, 19, 0, 2, 0, 0, 21, 37, 19,
    0, 36, 0, 1, 0, 0, 0, 0, 0, 4, 0, 331, 45, 343, 115, 540, 57, 180, 163, 198, 4, 41, 135, 78, 326,
    301, 187, 22, 211, 130, 324, 61, 38, 125, 41, 22, 36, 0, 0, 0, 0,
]

SEED_NORTH_STAR = 0x6D696E6871  # "minhq"
SEED_ZIPF = 0x7A697066          # "zipf"
SEED_ADV = 0x616476             # "adv"
_BYTE_STREAM_XOR = 0xB7E151628AED2A6A

_GAMMA = np.uint64(0x9E3779B97F4A7C15)
_M1 = np.uint64(0xBF58476D1CE4E5B9)
_M2 = np.uint64(0x94D049BB133111EB)


def splitmix64(seed: int, count: int, start: int = 0) -> np.ndarray:
    """Values start..start+count-1 of the splitmix64 sequence seeded by `seed`."""
    with np.errstate(over="ignore"):
        idx = np.arange(start + 1, start + count + 1, dtype=np.uint64)
        z = np.uint64(seed & 0xFFFFFFFFFFFFFFFF) + idx * _GAMMA
        z = (z ^ (z >> np.uint64(30))) * _M1
        z = (z ^ (z >> np.uint64(27))) * _M2
        return z ^ (z >> np.uint64(31))


def _unit(r: np.ndarray) -> np.ndarray:
    return (r >> np.uint64(11)).astype(np.float64) * (1.0 / (1 << 53))


def byte_alphabet(dist: str) -> Tuple[np.ndarray, np.ndarray]:
    """(symbols u8[], cumulative probabilities f64[]) for a byte distribution."""
    if dist == "hdr":
        syms = np.arange(0x20, 0x7F, dtype=np.uint8)
        w = np.asarray(NETBSD_HIST, dtype=np.float64) + 1.0
    elif dist == "print":
        syms = np.arange(0x20, 0x7F, dtype=np.uint8)
        w = np.ones(len(syms))
    elif dist == "adv":
        from .hc import code_table  # the kernels' own table (hc/huffmantable.go)

        lens, _ = code_table()
        syms = np.asarray([s for s in range(256) if lens[s] >= 26], dtype=np.uint8)
        w = np.ones(len(syms))
    else:
        raise ValueError(dist)
    cdf = np.cumsum(w / w.sum())
    cdf[-1] = 1.0
    return syms, cdf


def lengths(kind: str, n: int, seed: int, lo: int = 8, hi: int = 56) -> np.ndarray:
    r = splitmix64(seed, n)
    if kind == "uniform":
        span = np.uint64(hi - lo + 1)
        return (np.uint64(lo) + r % span).astype(np.int64)
    if kind == "fixed":
        return np.full(n, lo, dtype=np.int64)
    if kind == "clustered":  # blocks of 512 literals alternating U{lo..hi} and U{8..lo} (the packed encode's ranges over and under its staging)
        odd = (np.arange(n) // 512) % 2 == 1
        a = np.uint64(lo) + r % np.uint64(hi - lo + 1)
        b = np.uint64(8) + r % np.uint64(lo - 8 + 1)
        return np.where(odd, b, a).astype(np.int64)
    if kind == "zipf":  # P(L=k) ~ 1/(k-3), k in 4..256
        ks = np.arange(4, 257)
        cdf = np.cumsum(1.0 / (ks - 3))
        cdf /= cdf[-1]
        return ks[np.searchsorted(cdf, _unit(r), side="right").clip(0, len(ks) - 1)].astype(np.int64)
    raise ValueError(kind)


@dataclass
class Batch:
    data: np.ndarray  # u8, literals back to back
    off: np.ndarray   # u64, n+1
    name: str

    @property
    def n(self) -> int:
        return len(self.off) - 1

    @property
    def nbytes(self) -> int:
        return int(self.off[-1] - self.off[0])


def make_batch(n: int, length_kind: str = "uniform", dist: str = "hdr", seed: int = SEED_NORTH_STAR,
               lo: int = 8, hi: int = 56, name: str = "") -> Batch:
    L = lengths(length_kind, n, seed, lo, hi)
    off = np.zeros(n + 1, dtype=np.uint64)
    off[1:] = np.cumsum(L, dtype=np.uint64)
    total = int(off[-1])
    syms, cdf = byte_alphabet(dist)
    data = np.empty(total, dtype=np.uint8)
    chunk = 1 << 24
    for a in range(0, total, chunk):
        b = min(total, a + chunk)
        u = _unit(splitmix64(seed ^ _BYTE_STREAM_XOR, b - a, start=a))
        data[a:b] = syms[np.searchsorted(cdf, u, side="right").clip(0, len(syms) - 1)]
    return Batch(data, off, name or f"{n}x{length_kind}[{lo},{hi}]/{dist}")


# BASELINE.json configs as concrete batches.
def count_label(n: int) -> str:
    """2^20 -> "1M", 4*2^20 -> "4M", 2^16 -> "64K"; other sizes as digits."""
    if n and n % (1 << 20) == 0:
        return f"{n >> 20}M"
    if n and n % (1 << 10) == 0:
        return f"{n >> 10}K"
    return str(n)


def north_star(n: int = 1 << 20) -> Batch:
    return make_batch(n, "uniform", "hdr", SEED_NORTH_STAR, 8, 56, f"northstar-{count_label(n)}x U{{8..56}} hdr")


def config2(n: int = 1 << 20, dist: str = "hdr") -> Batch:
    return make_batch(n, "uniform", dist, SEED_NORTH_STAR, 8, 64, f"config2-{count_label(n)}x U{{8..64}} {dist}")


def config4(n: int = 1 << 24) -> Batch:
    return make_batch(n, "zipf", "hdr", SEED_ZIPF, name=f"config4-{count_label(n)}x zipf{{4..256}} hdr")


def config5(n: int = 4 << 20) -> Batch:
    return make_batch(n, "fixed", "adv", SEED_ADV, 128, 128, f"config5-{count_label(n)}x128B adv")


def config3(n: int = 1 << 20) -> Batch:
    """BASELINE.json configs[2]: the string literals of the reference's QIF
    header sets -- the netbsd.qif fields (names and values) and the literals
    embedded in hc/testcases_test.go / hc/qpack_test.go, as extracted into
    tests/golden/ -- tiled to n literals."""
    import json
    import os

    g = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tests", "golden")
    with open(os.path.join(g, "netbsd_qif.json")) as f:
        fields = json.load(f)["fields"]
    with open(os.path.join(g, "embedded_literals.json")) as f:
        embedded = json.load(f)
    lits = []
    for fl in fields:
        if fl:
            lits += [fl[0].encode(), fl[1].encode()]
    lits += [r["text"].encode() for r in embedded]
    reps = n // len(lits) + 1
    tiled = (lits * reps)[:n]
    L = np.fromiter((len(x) for x in tiled), dtype=np.uint64, count=n)
    off = np.zeros(n + 1, dtype=np.uint64)
    off[1:] = np.cumsum(L, dtype=np.uint64)
    data = np.frombuffer(b"".join(tiled), dtype=np.uint8).copy()
    return Batch(data, off, f"config3-{count_label(n)}x qif corpus tiled")


# ---- the same batches generated on a device (torch) ------------------------
# Bit-identical to make_batch: splitmix64 in wrapping int64 arithmetic
# (logical shifts by masking), the same float64 unit values and CDFs.  Used for
# the full-size configs (2^24 literals), which numpy builds in minutes.
def _splitmix64_t(torch, seed: int, count: int, start: int, device):
    idx = torch.arange(start + 1, start + count + 1, dtype=torch.int64, device=device)

    def s64(x):  # an unsigned 64-bit constant as the int64 with the same bits
        x &= 0xFFFFFFFFFFFFFFFF
        return x - (1 << 64) if x >= (1 << 63) else x

    def shr(z, k):  # logical right shift
        return (z >> k) & ((1 << (64 - k)) - 1)

    z = idx * s64(0x9E3779B97F4A7C15) + s64(seed)
    z = (z ^ shr(z, 30)) * s64(0xBF58476D1CE4E5B9)
    z = (z ^ shr(z, 27)) * s64(0x94D049BB133111EB)
    return z ^ shr(z, 31)


def _unit_t(torch, r):
    return ((r >> 11) & ((1 << 53) - 1)).to(torch.float64) * (1.0 / (1 << 53))


def make_batch_device(n: int, length_kind: str = "uniform", dist: str = "hdr", seed: int = SEED_NORTH_STAR,
                      lo: int = 8, hi: int = 56, device="cuda", chunk: int = 1 << 26):
    """make_batch's literals as device tensors (data u8, off int64[n+1])."""
    import torch

    r = _splitmix64_t(torch, seed, n, 0, device)
    if length_kind == "uniform":
        span = hi - lo + 1
        rh, rl = (r >> 32) & 0xFFFFFFFF, r & 0xFFFFFFFF  # unsigned r mod span, in int64
        L = lo + ((rh % span) * ((1 << 32) % span) + rl % span) % span
    elif length_kind == "fixed":
        L = torch.full((n,), lo, dtype=torch.int64, device=device)
    elif length_kind == "zipf":
        ks = np.arange(4, 257)
        cdf = np.cumsum(1.0 / (ks - 3))
        cdf /= cdf[-1]
        i = torch.searchsorted(torch.from_numpy(cdf).to(device), _unit_t(torch, r), right=True)
        L = torch.from_numpy(ks).to(device)[i.clamp(0, len(ks) - 1)]
    else:
        raise ValueError(length_kind)
    del r
    off = torch.zeros(n + 1, dtype=torch.int64, device=device)
    torch.cumsum(L, 0, out=off[1:])
    total = int(off[-1].item())
    syms, cdf = byte_alphabet(dist)
    syms_t, cdf_t = torch.from_numpy(syms).to(device), torch.from_numpy(cdf).to(device)
    data = torch.empty(total, dtype=torch.uint8, device=device)
    for a in range(0, total, chunk):
        b = min(total, a + chunk)
        u = _unit_t(torch, _splitmix64_t(torch, seed ^ _BYTE_STREAM_XOR, b - a, a, device))
        data[a:b] = syms_t[torch.searchsorted(cdf_t, u, right=True).clamp(0, len(syms) - 1)]
    return data, off
