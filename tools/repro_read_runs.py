#!/usr/bin/env python3
"""Reproducer: tests/test_strings.py::test_read_gaps_and_order[runs]'s block
through mhq_read_strings once, every string checked against the oracle.
Prints one JSON line.  (Run under a time limit; MHQ_LIB_PATH picks a build.)
"""
import json
import os
import random
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from minhq_amd import hc  # noqa: E402
from oracle import oracle  # noqa: E402


def _random_strings(rng, n):  # tests/test_strings.py's generator
    alpha = b"abcdefghijklmnopqrstuvwxyz0123456789-_./:;=, "
    out = []
    for _ in range(n):
        kind = rng.random()
        L = rng.choice([0, 1, 2, 5, 30, 126, 127, 128, 200, 300]) if kind < 0.3 else rng.randint(0, 60)
        if rng.random() < 0.8:
            out.append(bytes(rng.choice(alpha) for _ in range(L)))
        else:
            out.append(bytes(rng.randrange(256) for _ in range(L)))
    return out


def main():
    order = sys.argv[1] if len(sys.argv) > 1 else "runs"
    rng = random.Random({"in_order": 31, "shuffled": 32, "runs": 33}[order])
    strs = _random_strings(rng, 20000)
    blk, pos, prefixes = bytearray(), [], []
    for s in strs:
        blk += bytes(rng.randrange(256) for _ in range(rng.choice([0, 0, 1, 3, 9])))
        p = rng.choice([7, 5, 3])
        pos.append(len(blk))
        prefixes.append(p)
        blk += oracle.write_string(s, prefix=p, choice=rng.choice([1, 1, 1, 2, 0]),
                                   lead=rng.randrange(1 << (7 - p)) if p < 7 else 0, lead_bits=7 - p)
    blk = bytes(blk)
    idx = list(range(len(strs)))
    if order == "shuffled":
        rng.shuffle(idx)
    elif order == "runs":
        runs = [idx[k:k + 300] for k in range(0, len(idx), 300)]
        rng.shuffle(runs)
        idx = [i for r in runs for i in r]
    P = [pos[i] for i in idx]
    F = [prefixes[i] for i in idx]
    refs = []
    for i in idx:
        ref, rc, used = oracle.read_string(blk[pos[i]:pos[i] + 4096], prefix=prefixes[i], skip_bits=7 - prefixes[i])
        refs.append((ref, {0: 0, 1: 1, -1: 2}[rc], pos[i] + used))
    codec = hc.Codec(1)
    bad = 0
    for rep in range(3):
        vals, st, nxt = codec.read_strings(blk, P, F)
        for k in range(len(idx)):
            if (vals[k], int(st[k]), int(nxt[k])) != refs[k]:
                bad += 1
    print(json.dumps({"order": order, "strings": len(idx), "mismatches": bad}), flush=True)
    codec.close()


if __name__ == "__main__":
    main()
