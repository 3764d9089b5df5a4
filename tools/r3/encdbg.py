"""Debug: the coop encode on one batch, mismatch runs against the oracle."""
import random
import sys

import numpy as np
import torch

sys.path.insert(0, ".")
from minhq_amd import hc  # noqa: E402
from oracle import oracle  # noqa: E402


def runs(got, ref):
    d = np.nonzero(got != ref)[0]
    out = []
    for x in d:
        if out and x == out[-1][1]:
            out[-1][1] = x + 1
        else:
            out.append([int(x), int(x) + 1])
    return out


def check(name, lits, c):
    data, off = hc.pack(lits)
    el = oracle.encode_len_batch(data, off)
    eoff = np.zeros(len(el) + 1, dtype=np.uint64)
    eoff[1:] = np.cumsum(el)
    ref = oracle.encode_batch(data, off, eoff)
    d = torch.from_numpy(np.concatenate([data, np.zeros(64, np.uint8)])).cuda()
    o = torch.from_numpy(off.astype(np.int64)).cuda()
    eo = torch.from_numpy(eoff.astype(np.int64)).cuda()
    out = torch.full((int(eoff[-1]) + 64,), 0x5A, dtype=torch.uint8, device="cuda")
    c.encode_dev(d, o, out, eo)
    torch.cuda.synchronize()
    got = out.cpu().numpy()[: int(eoff[-1])]
    r = runs(got, ref)
    print(name, "n", len(lits), "bytes", int(eoff[-1]), "mismatch runs", len(r), flush=True)
    for a, b in r[:12]:
        lit = int(np.searchsorted(eoff, a, side="right")) - 1
        print("   [%d,%d) lit %d wave %d eoff %d..%d got %s want %s" % (
            a, b, lit, lit // 64, int(eoff[lit]), int(eoff[lit + 1]), got[a:min(b, a + 6)].tobytes().hex(),
            ref[a:min(b, a + 6)].tobytes().hex()), flush=True)
    tail = got[int(eoff[-1]):]


def main():
    c = hc.Codec()
    rng = random.Random(99)
    lits = [bytes(rng.randrange(256) for _ in range(rng.randrange(0, 90))) for _ in range(5000)]
    check("rand99", lits, c)
    check("rand99[:64]", lits[:64], c)
    check("rand99[:128]", lits[:128], c)
    rng = random.Random(5)
    check("ascii", [bytes(rng.randrange(32, 127) for _ in range(rng.randrange(0, 90))) for _ in range(3000)], c)
    check("one_long", [bytes(rng.randrange(256) for _ in range(5000))], c)
    check("ones", [bytes([255] * 3000)], c)
    check("zeros", [bytes([48] * 3000)], c)


main()
