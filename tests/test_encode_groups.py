"""The wave-cooperative encode (huff_encode.hip encode_coop_kernel) with each
literal-group count K a wave can take (K groups of 64 literals share one
stream of 1-KiB rounds).  The launch picks K from the batch size, so small
test batches would only ever see K = 1: here every K is forced through
MHQ_ENC_K in a child process (one process at a time on the GPU) and checked
against the oracle (oracle/huff_oracle.c, the restated hc/huffman.go:23-37
Write + Pad) on batches that stress the round/mark logic: random bytes (long
codes), tiny and empty literals (many starts per 16-B chunk), long literals
beside short ones, unaligned input and output bases, output regions with
slack, a partial last group, empty regions (the fallback path), and a
batch of 1.35 M literals: more ranges than the cooperative kernel's
resident grid holds.
"""
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

CHILD = r'''
import os, random, sys
import numpy as np, torch
THREAD = os.environ.get("MHQ_ENC_FORM") == "thread"
sys.path.insert(0, ".")
from minhq_amd import hc
from oracle import oracle

c = hc.Codec()

def run(lits, ibias=0, obias=0, slack=None, skip=None, seed=0):
    data, off = hc.pack(lits)
    n = len(lits)
    el = oracle.encode_len_batch(data, off)
    reg = el.astype(np.uint64)
    if slack is not None:
        reg = reg + slack.astype(np.uint64)
    if skip is not None:
        reg = np.where(skip, 0, reg).astype(np.uint64)
    eoff = np.zeros(n + 1, dtype=np.uint64); eoff[1:] = np.cumsum(reg)
    exact = np.zeros(n + 1, dtype=np.uint64); exact[1:] = np.cumsum(el)
    ref = oracle.encode_batch(data, off, exact)
    d = torch.zeros(len(data) + ibias + 64, dtype=torch.uint8)
    d[ibias:ibias + len(data)] = torch.from_numpy(data)
    o = torch.from_numpy((off + np.uint64(ibias)).astype(np.int64))
    eo = torch.from_numpy((eoff + np.uint64(obias)).astype(np.int64))
    out = torch.full((int(eoff[-1]) + obias + 64,), 0x5A, dtype=torch.uint8, device="cuda")
    c.encode_dev(d.cuda(), o.cuda(), out, eo.cuda())
    torch.cuda.synchronize()
    got = out.cpu().numpy()
    assert (got[:obias] == 0x5A).all() and (got[obias + int(eoff[-1]):] == 0x5A).all(), "wrote outside the regions"
    for i in range(n):
        g0 = obias + int(eoff[i])
        if reg[i] == 0:
            continue
        r = ref[int(exact[i]):int(exact[i + 1])]
        assert got[g0:g0 + len(r)].tobytes() == r.tobytes(), ("literal", i, n)
        # (bytes past enc_len are unspecified, mhq_huff.h; the cooperative
        # kernel's complemented ring leaves them all ones)
        if not THREAD:
            assert (got[g0 + len(r):g0 + int(reg[i])] == 0xFF).all(), ("slack", i)

rng = random.Random(99)
run([bytes(rng.randrange(256) for _ in range(rng.randrange(0, 90))) for _ in range(5000)])
rng = random.Random(3)
tiny = [bytes(rng.randrange(32, 127) for _ in range(rng.randrange(0, 6))) for _ in range(20000)]
run(tiny, ibias=5, obias=9)
mixed = []
for i in range(3000):
    k = rng.randrange(10)
    L = rng.randrange(500, 3000) if k == 0 else (0 if k == 1 else rng.randrange(1, 40))
    mixed.append(bytes(rng.randrange(256) if rng.random() < 0.3 else rng.randrange(32, 127) for _ in range(L)))
run(mixed, ibias=3, obias=1)
run(mixed[:64 * 8 * 4 * 3 + 37], ibias=15, obias=15)
nr = np.random.default_rng(1)
run(tiny[:9000], slack=nr.integers(0, 4, 9000))
skip = nr.random(9000) < 0.01
run(tiny[:9000], skip=skip)
run([bytes([255] * 4000), b"a", bytes(range(256)) * 7])
# more ranges than the cooperative kernel's resident grid holds (1,024
# workgroups x 4 waves): every wave loops over several ranges
big = np.random.default_rng(7)
nbig = (1 << 20) + 300000
lens = big.integers(0, 48, nbig)
blob = big.integers(32, 127, int(lens.sum()), dtype=np.uint8).tobytes()
cuts = np.concatenate([[0], np.cumsum(lens)])
run([blob[cuts[i]:cuts[i + 1]] for i in range(nbig)], ibias=7, obias=3)
print("ok")
'''


@pytest.mark.gpu
@pytest.mark.parametrize("k", [1, 2, 4, 8, "thread"])
def test_encode_literal_groups(k):
    # "thread": the thread-per-literal kernel for every batch (MHQ_ENC_FORM),
    # which the launch otherwise picks only for batches of short literals
    env = dict(os.environ, MHQ_ENC_FORM="thread") if k == "thread" else dict(os.environ, MHQ_ENC_K=str(k))
    r = subprocess.run([sys.executable, "-c", CHILD], env=env, cwd=ROOT, capture_output=True, text=True,
                       timeout=240)
    assert r.returncode == 0 and "ok" in r.stdout, r.stdout[-3000:] + r.stderr[-3000:]
