#!/usr/bin/env python3
"""Host-side cost of the bench step (GPU box): how long the CPU takes to
enqueue bench.py's round trips (encode_layout_dev, encode_dev, decode_dev
through ctypes), against the GPU time per step.  Prints one JSON line.

    python3 tools/host_overhead.py [--steps 200] [--streams 4]
"""
import argparse
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

import bench  # noqa: E402
from minhq_amd import hc, workloads  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--steps", type=int, default=200)
    ap.add_argument("--streams", type=int, default=4)
    args = ap.parse_args()
    dev = torch.device("cuda:0")
    codec = hc.Codec(devices=[0])
    batch = workloads.config2(1 << 20, "hdr")
    enc_b, cap_b = bench.encoded_sizes(codec, batch, dev)
    slots = [bench.Slot(batch, enc_b, cap_b, dev) for _ in range(8)]
    streams = [torch.cuda.Stream(device=dev).cuda_stream for _ in range(args.streams)]
    for i, s in enumerate(slots):
        bench.round_trip(codec, s, streams[i % len(streams)])
    torch.cuda.synchronize()
    res = {}
    for name, fn in (
        ("layout", lambda s, st: codec.encode_layout_dev(s.data, s.off, s.enc_len, s.enc_off, s.cap_off, stream=st)),
        ("encode", lambda s, st: codec.encode_dev(s.data, s.off, s.enc, s.enc_off, stream=st)),
        ("decode", lambda s, st: codec.decode_dev(s.enc, s.enc_off, s.out, s.cap_off, s.out_len, s.status,
                                                  stream=st)),
        ("round_trip", lambda s, st: bench.round_trip(codec, s, st)),
    ):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for i in range(args.steps):
            fn(slots[i % len(slots)], streams[i % len(streams)])
        t1 = time.perf_counter()
        torch.cuda.synchronize()
        t2 = time.perf_counter()
        res[name] = {"enqueue_us_per_call": round((t1 - t0) / args.steps * 1e6, 2),
                     "wall_us_per_call": round((t2 - t0) / args.steps * 1e6, 2)}
    print(json.dumps(res), flush=True)
    codec.close()


if __name__ == "__main__":
    main()
