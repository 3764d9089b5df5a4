#!/usr/bin/env python3
"""Decode forms side by side: the tile kernel and the streamed decode.

    python tools/decode_ab.py --configs northstar,config2,config3 --forms tile,stream --iters 30

For each config: encodes the batch on the device, then per form decodes it
`--iters` times back to back over rotating buffer copies (HIP events around
the run, as bench.py's decode_only), checks every decoded byte, length and
status against the plaintext, and prints one line (us per launch, fraction of
the HBM roofline on SURVEY §8d's algorithmic bytes).  The forms are switched
with mhq_set_decode_form (include/mhq_huff.h).
"""
from __future__ import annotations

import argparse
import json
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

FORMS = {"auto": 0, "tile": 1, "stream": 2}


def diag_report(L):
    """Summarises the MHQ_DIAG_STREAM counters of the last launch."""
    import ctypes

    K = 16
    buf = (ctypes.c_ulonglong * (1024 * 16 * K))()
    L.mhq_diag_stream.restype = ctypes.c_int
    L.mhq_diag_stream(buf, 1024 * 16 * K)
    a = np.frombuffer(buf, dtype=np.uint64).reshape(1024, 16, K).astype(np.float64)
    dec = a[:, :12, :].reshape(-1, K)
    dec = dec[dec[:, 0] > 0]
    ld = a[:, 12:, :].reshape(-1, K)
    ld = ld[ld[:, 8] > 0]
    f = lambda x: f"{x:.0f}"  # noqa: E731
    print(f"  decoders {len(dec)}: cycles {f(dec[:, 0].mean())} (max {f(dec[:, 0].max())}) service "
          f"{f(dec[:, 1].mean())} wait {f(dec[:, 2].mean())} | services {dec[:, 3].mean():.1f} groups "
          f"{dec[:, 4].mean():.1f} active lanes/group {(dec[:, 5] / np.maximum(dec[:, 4], 1)).mean():.1f} "
          f"assigned/service {(dec[:, 6] / np.maximum(dec[:, 3], 1)).mean():.1f} flushes {dec[:, 7].mean():.1f}",
          file=sys.stderr, flush=True)
    print(f"  loaders {len(ld)}: cycles {f(ld[:, 8].mean())} iterations {ld[:, 9].mean():.1f} vmcnt-wait "
          f"{f(ld[:, 10].mean())} chunks {ld[:, 11].mean():.1f} idle iterations {ld[:, 12].mean():.1f}",
          file=sys.stderr, flush=True)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--configs", default="northstar,config2,config3,config2print")
    ap.add_argument("--forms", default="tile,stream")
    ap.add_argument("--iters", type=int, default=30)
    ap.add_argument("--reps", type=int, default=3, help="timed runs per form (median reported)")
    ap.add_argument("--rotate-gib", type=float, default=1.0)
    ap.add_argument("--n", type=int, default=0)
    ap.add_argument("--diag", action="store_true", help="a -DMHQ_DIAG_STREAM build (MHQ_LIB_PATH): per-wave counters")
    ap.add_argument("--sized", action="store_true", help="decode through mhq_huff_decode_sized_dev (the long-literal form for long batches)")
    args = ap.parse_args()

    import torch

    import bench
    from minhq_amd import _lib, hc
    from tools.kernel_driver import batch_for

    L = _lib.load()
    dev = torch.device("cuda:0")
    codec = hc.Codec(devices=[0])
    for cfg in args.configs.split(","):
        b = batch_for(cfg, args.n)
        data = torch.from_numpy(b.data).to(dev)
        off = torch.from_numpy(b.off.view(np.int64)).to(dev)
        dv = bench.Dev(codec, data, off, dev)
        slots = bench.decode_slots(dv, 0, b.n, args.rotate_gib * (1 << 30), dev)
        alg = bench.decode_algorithmic_bytes(b.n, dv.enc_bytes, b.nbytes)
        for form in args.forms.split(","):
            L.mhq_set_decode_form(FORMS[form])

            def run(i):
                s = slots[i % len(slots)]
                codec.decode_dev(s.enc, s.enc_off, s.out, s.cap_off, s.out_len, s.status,
                                 in_bytes=dv.enc_bytes if args.sized else 0)

            for s in slots[:2]:
                s.out.zero_()
            run(0)
            ok = True
            try:
                bench.check_decode(dv, 0, b.n, slots[0])
            except AssertionError as e:
                ok = str(e)
            for i in range(3):
                run(i)
            times = sorted(bench.events_ms(run, args.iters) for _ in range(args.reps))
            ms = times[len(times) // 2]
            if args.diag and form == "stream":
                run(0)
                torch.cuda.synchronize()
                diag_report(L)
            print(json.dumps({"config": cfg, "form": form, "n": b.n, "us": round(ms * 1e3, 2),
                              "us_all": [round(t * 1e3, 2) for t in times],
                              "hbm_frac": round(alg / (ms / 1e3) / 1e9 / bench.HBM_PEAK_GBS, 4),
                              "check": ok}), flush=True)
        del slots, dv
        torch.cuda.empty_cache()
    L.mhq_set_decode_form(0)


if __name__ == "__main__":
    main()
