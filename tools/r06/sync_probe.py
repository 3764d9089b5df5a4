#!/usr/bin/env python3
"""Where the short bench's extra microseconds go: bench.py's step loop (the
same slots, streams and bound calls), timed as host submission, then the
closing torch.cuda.synchronize(), for K-step runs repeated.

    python tools/r06/sync_probe.py --steps 20 --reps 10
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--reps", type=int, default=10)
    ap.add_argument("--long", type=int, default=2000)
    ap.add_argument("--streams", default="4", help="comma-separated stream counts to try")
    ap.add_argument("--chain", default="0", help="comma-separated: 1 = each step's encode waits for the previous step's encode (an event)")
    args = ap.parse_args()

    import torch

    import bench
    from minhq_amd import hc, workloads

    bench.PACKED = True
    dev = torch.device("cuda", 0)
    codec = hc.Codec(devices=[0])
    batch = workloads.make_batch(1 << 20, "uniform", "hdr", workloads.SEED_NORTH_STAR, 8, 64, "config2")
    enc_b, cap_b = bench.encoded_sizes(codec, batch, dev)
    first = bench.Slot(batch, enc_b, cap_b, dev, True)
    R = max(2, int(np.ceil(bench.GIB / first.nbytes())))
    R += (-R) % 12
    slots = [first] + [bench.Slot(batch, enc_b, cap_b, dev, True) for _ in range(R - 1)]
    for s in slots:
        bench.round_trip(codec, s)
        bench.verify_slot(s)
    all_streams = [torch.cuda.Stream(device=dev).cuda_stream for _ in range(4)]
    import ctypes as C

    hip = C.CDLL("libamdhip64.so")
    hip.hipEventCreateWithFlags.argtypes = [C.POINTER(C.c_void_p), C.c_uint]
    hip.hipEventRecord.argtypes = [C.c_void_p, C.c_void_p]
    hip.hipStreamWaitEvent.argtypes = [C.c_void_p, C.c_void_p, C.c_uint]
    evs = [C.c_void_p() for _ in range(4)]
    for e in evs:
        assert hip.hipEventCreateWithFlags(C.byref(e), 2) == 0
    for chain in [int(x) for x in args.chain.split(",")]:
        for S in [int(x) for x in args.streams.split(",")]:
            streams = all_streams[:S]
            bound = [bench.bind_round_trip(codec, slots[i], streams[i % S]) for i in range(R)]
            if chain:
                bound = [chained(hip, evs, bound[i], streams[i % S], i) for i in range(R)]
            probe(args, torch, bench, codec, slots, streams, bound, R, S, chain)
    codec.close()


def chained(hip, evs, calls, stream, i):
    """Step i's calls with its encode after step i - 1's (stream i % S waits
    for the event recorded after the previous step's encode)."""
    enc, dec = calls
    wait_ev, rec_ev = evs[(i - 1) % len(evs)], evs[i % len(evs)]
    # (R is a multiple of len(evs): slot i's events are the same on every pass)
    return (lambda: hip.hipStreamWaitEvent(stream, wait_ev, 0), enc, lambda: hip.hipEventRecord(rec_ev, stream), dec)


def probe(args, torch, bench, codec, slots, streams, bound, R, S, chain=0):

    def run(k, warm=5):
        for i in range(warm):
            bench.round_trip(codec, slots[i % R], streams[i % S], bound[i % R])
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for i in range(k):
            bench.round_trip(codec, slots[i % R], streams[i % S], bound[i % R])
        t1 = time.perf_counter()
        torch.cuda.synchronize()
        t2 = time.perf_counter()
        return (t1 - t0) * 1e6, (t2 - t0) * 1e6

    out = []
    for rep in range(args.reps):
        sub, tot = run(args.steps)
        out.append((sub, tot))
    sub = np.array([o[0] for o in out])
    tot = np.array([o[1] for o in out])
    _, tot_long = run(args.long)
    res = {"streams": S, "chain": chain, "steps": args.steps, "submit_us_med": round(float(np.median(sub)), 1),
           "submit_us_per_step": round(float(np.median(sub)) / args.steps, 2),
           "total_us_med": round(float(np.median(tot)), 1),
           "us_per_step_med": round(float(np.median(tot)) / args.steps, 2),
           "us_per_step_all": [round(t / args.steps, 2) for t in tot],
           "long_us_per_step": round(tot_long / args.long, 2),
           "fixed_overhead_us": round(float(np.median(tot)) - args.steps * tot_long / args.long, 1)}
    print(json.dumps(res), flush=True)
    # a single step, and an empty synchronize, for scale
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    torch.cuda.synchronize()
    t1 = time.perf_counter()
    one = [run(1)[1] for _ in range(10)]
    print(json.dumps({"empty_sync_us": round((t1 - t0) * 1e6, 1), "one_step_us_med": round(float(np.median(one)), 1)}),
          flush=True)


if __name__ == "__main__":
    main()
