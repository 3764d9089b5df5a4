"""The look-backs' way out of an unscheduled predecessor:
with MHQ_PK_HELP_POLLS=0 every predecessor a look-back finds unpublished is
computed by the waiter itself -- the packed encode's workgroup sizes the
stuck range and publishes its aggregate for it (enc_packed.hip), the read
fallback's thread parses the stuck workgroup's frames (read_strings.hip
range_cap_sum) -- so the help path, which a normal run only takes when the
dispatcher starves a predecessor, runs on every call.  In a child process
(the setting is read once per process), against the oracle: packed encodes
of many ranges on one and on four streams, and read_strings over shuffled
strings (the fallback's look-back)."""
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

CHILD = r'''
import random, sys
import numpy as np, torch
sys.path.insert(0, ".")
from minhq_amd import hc, workloads as w
from oracle import oracle

c = hc.Codec()
dev = torch.device("cuda:0")
streams = [None] + [torch.cuda.Stream().cuda_stream for _ in range(3)]

def encode(b, k):
    n, in_bytes = b.n, int(b.off[-1])
    t_data = torch.from_numpy(b.data.copy()).to(dev)
    t_off = torch.from_numpy(b.off.view(np.int64).copy()).to(dev)
    enc_len = torch.full((n,), -1, dtype=torch.int32, device=dev)
    out_off = torch.full((n + 1,), -1, dtype=torch.int64, device=dev)
    cap_off = torch.full((n + 1,), -1, dtype=torch.int64, device=dev)
    out = torch.full((30 * in_bytes // 8 + n,), 0xA5, dtype=torch.uint8, device=dev)
    torch.cuda.synchronize()
    c.encode_packed_dev(t_data, t_off, in_bytes, enc_len, out_off, cap_off, out, base=k, stream=streams[k % 4])
    return enc_len, out_off, cap_off, out

for n in (1 << 20, 70000):
    b = w.north_star(n)
    calls = [encode(b, k) for k in range(4)]
    torch.cuda.synchronize()
    ref_len = oracle.encode_len_batch(b.data, b.off, nthreads=8)
    eoff = np.zeros(n + 1, dtype=np.uint64); eoff[1:] = np.cumsum(ref_len, dtype=np.uint64)
    coff = np.zeros(n + 1, dtype=np.uint64); coff[1:] = np.cumsum(ref_len.astype(np.uint64) * 8 // 5)
    ref = oracle.encode_batch(b.data, b.off, eoff, nthreads=8).tobytes()
    for k, (enc_len, out_off, cap_off, out) in enumerate(calls):
        assert np.array_equal(enc_len.cpu().numpy().view(np.uint32), ref_len), (n, k)
        assert np.array_equal(out_off.cpu().numpy().view(np.uint64), eoff + k), (n, k)
        assert np.array_equal(cap_off.cpu().numpy().view(np.uint64), coff + k), (n, k)
        assert out.cpu().numpy()[: int(eoff[-1])].tobytes() == ref, (n, k)

rng = random.Random(21)
alpha = b"abcdefghijklmnopqrstuvwxyz0123456789-_./:;=, "
strs = [bytes(rng.choice(alpha) for _ in range(rng.randint(0, 60))) for _ in range(60000)]
blk, pos = bytearray(), []
for s in strs:
    pos.append(len(blk))
    blk += oracle.write_string(s, prefix=7, choice=rng.choice([0, 1, 1, 2]))
blk = bytes(blk)
idx = list(range(len(strs)))
rng.shuffle(idx)
P = [pos[i] for i in idx]
vals, st, nxt = c.read_strings(blk, P, [7] * len(P))
for j, i in enumerate(idx):
    ref, rc, used = oracle.read_string(blk[pos[i]:], prefix=7)
    assert vals[j] == ref and int(nxt[j]) == pos[i] + used, j
print("ok")
'''


@pytest.mark.gpu
def test_lookbacks_with_forced_help():
    env = dict(os.environ, MHQ_PK_HELP_POLLS="0")
    r = subprocess.run([sys.executable, "-c", CHILD], env=env, cwd=ROOT, capture_output=True, text=True, timeout=240)
    assert r.returncode == 0 and "ok" in r.stdout, r.stdout[-3000:] + r.stderr[-3000:]
