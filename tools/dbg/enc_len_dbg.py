import os, sys, random
sys.path.insert(0, os.getcwd())
import numpy as np
from minhq_amd import hc, build
from oracle import oracle
oracle.build()
rng = random.Random(99)
lits = [bytes(rng.randrange(256) for _ in range(rng.randrange(0, 90))) for _ in range(5000)]
data, off = hc.pack(lits)
codec = hc.Codec(devices=[0])
got = codec.encode_len(data, off)
ref = np.array([oracle.encoded_len(l) for l in lits])
bad = np.nonzero(got != ref)[0]
print("mismatches", len(bad), "first", bad[:20])
for i in bad[:10]:
    print(i, i % 64, (i // 64), len(lits[i]), got[i], ref[i])
