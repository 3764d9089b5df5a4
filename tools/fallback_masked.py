#!/usr/bin/env python3
"""read_strings' out-of-order fallback when its grid cannot be resident at once.

Run with the process's queues limited to a few CUs (HSA_CU_MASK), so that
the fallback kernel's grid (one workgroup per CU of the device) cannot be
resident at once: its workgroups wait only for lower-numbered ones (the
decoupled look-back), so the call completes with the same results as without
the mask.  Prints one JSON line (status counts and checksums of the strings
and next positions, to compare between a masked and an unmasked run).

    HSA_CU_MASK=0:0-31 python3 tools/fallback_masked.py
"""
import hashlib
import json
import os
import random
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import numpy as np  # noqa: E402
import torch  # noqa: E402

from minhq_amd import _lib, hc  # noqa: E402


def main():
    rng = random.Random(5)
    alpha = b"abcdefghijklmnopqrstuvwxyz0123456789-_./:;=, "
    n = 1 << 16
    codec = hc.Codec(devices=[0])
    lits = [bytes(rng.choice(alpha) for _ in range(rng.randint(1, 40))) for _ in range(n)]
    frames = codec.write_strings(lits, [7] * n, None, hc.HuffmanCodingAlways)
    pos = np.zeros(n, dtype=np.uint64)
    pos[1:] = np.cumsum([len(f) for f in frames])[:-1]
    blk = b"".join(frames)
    P = pos[::-1].copy()  # reverse block order: the fused pass sends the call to the fallback
    dev = torch.device("cuda:0")
    t_blk = torch.frombuffer(bytearray(blk), dtype=torch.uint8).to(dev)
    t_pos = torch.from_numpy(P.view(np.int64)).to(dev)
    t_lim = torch.full((n,), len(blk), dtype=torch.int64, device=dev)
    t_pf = torch.full((n,), 7, dtype=torch.uint8, device=dev)
    out = torch.zeros(len(blk) * 8 // 5 + 16, dtype=torch.uint8, device=dev)
    out_off = torch.zeros(n + 1, dtype=torch.int64, device=dev)
    out_len = torch.zeros(n, dtype=torch.int32, device=dev)
    st = torch.zeros(n, dtype=torch.uint8, device=dev)
    nxt = torch.zeros(n, dtype=torch.int64, device=dev)
    t0 = time.perf_counter()
    codec.read_strings_dev(t_blk, t_pos, t_lim, t_pf, out, out_off, out_len, st, nxt)
    torch.cuda.synchronize()
    dt = time.perf_counter() - t0
    s = st.cpu().numpy()
    counts = {int(k): int(v) for k, v in zip(*np.unique(s, return_counts=True))}
    oo, ol, o = out_off.cpu().numpy(), out_len.cpu().numpy(), out.cpu().numpy()
    got = [o[oo[k]:oo[k] + ol[k]].tobytes() for k in range(n)]
    order = {int(q): i for i, q in enumerate(pos)}
    print(json.dumps({"cu_mask": os.environ.get("HSA_CU_MASK", ""), "strings": n, "seconds": round(dt, 3),
                      "status_counts": counts, "ok": int(counts.get(_lib.MHQ_STR_OK, 0)),
                      "values_equal_written": got == [lits[order[int(q)]] for q in P],
                      "strings_sha": hashlib.sha256(b"\0".join(got)).hexdigest()[:16],
                      "next_sum": int(nxt.cpu().numpy().sum())}), flush=True)
    codec.close()


if __name__ == "__main__":
    main()
