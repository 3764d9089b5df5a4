#!/usr/bin/env python3
"""Host-memory (PCIe-inclusive) decode rate before and after the things a
long-lived caller does in between (a later decode in the
same process ran at 5-9 GiB/s instead of 23-24).

    python tools/hostpath.py [--steps a,b,...]

Times mhq_huff_decode of the config-2 batch (pinned input and outputs) three
times, then runs each disturbance in turn and times the decode again after
it.  Disturbances:
  devalloc  8 GiB of device memory allocated, touched and freed (torch, then
            empty_cache)
  devkeep   the same, without empty_cache (torch keeps the memory cached)
  smallfree 64 MiB of device memory allocated and freed (empty_cache)
  sleep     2 s idle
  pinalloc  2 GiB of pinned host memory allocated, touched and freed
  bigdec    config 5's host decode (4 x 2^20 x 128 B adversarial literals)
  lenbig    encode_len of the batch with 16 MB chunks (MHQ_HOST_LEN_CHUNK_MB
            is read once per process: run with it set in the environment)
  encode    the host encode (encode_len + host scan + encode) of the batch
  newctx    a second context opened, used and closed
  repin     (not a disturbance) the inputs and the output pool pinned afresh
  pageable  (not a disturbance) one decode into pageable outputs
Prints one JSON line: GiB/s per measurement, in order.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--steps", default="devalloc,sleep,pinalloc,devkeep,smallfree,encode,lenbig,bigdec,newctx")
    args = ap.parse_args()
    import torch

    import bench
    from minhq_amd import hc, workloads

    codec = hc.Codec(devices=[0])
    b = workloads.make_batch(1 << 20, "uniform", "hdr", workloads.SEED_NORTH_STAR, 8, 64, "config2")
    pin = lambda a: torch.from_numpy(a).pin_memory().numpy()  # noqa: E731
    data, off = pin(b.data), pin(b.off)
    epool, dpool = bench.PinnedPool(), bench.PinnedPool()
    enc, eoff = codec.encode(data, off, alloc=epool)
    enc, eoff = pin(np.array(enc)), pin(np.array(eoff))
    cap = pin(hc.capacity_offsets(eoff))

    S = {"enc": enc, "eoff": eoff, "cap": cap, "dpool": dpool}  # (replaced by the repin step)

    def dec():
        S["dpool"].rewind()
        t0 = time.perf_counter()
        _, _, out_len, st = codec.decode(S["enc"], S["eoff"], S["cap"], alloc=S["dpool"])
        t1 = time.perf_counter()
        assert not st.any() and np.array_equal(out_len.astype(np.uint64), np.diff(b.off))
        return round(b.nbytes / (t1 - t0) / (1 << 30), 2)

    bw_h = torch.empty(256 << 20, dtype=torch.uint8).pin_memory()  # (allocated once: pinning is itself a step)
    bw_d = torch.empty(256 << 20, dtype=torch.uint8, device="cuda")

    def rawbw():  # pinned host -> device and back, 256 MiB, torch copies
        h, d = bw_h, bw_d
        d.copy_(h, non_blocking=True)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        d.copy_(h, non_blocking=True)
        torch.cuda.synchronize()
        t1 = time.perf_counter()
        h.copy_(d, non_blocking=True)
        torch.cuda.synchronize()
        t2 = time.perf_counter()
        return {"h2d": round(0.25 / (t1 - t0), 2), "d2h": round(0.25 / (t2 - t1), 2)}

    res = {"first": [dec() for _ in range(4)], "rawbw_first": rawbw()}
    # the host scan over encode_len's output: pinned vs pageable (hc.encode)
    lens_pg = codec.encode_len(data, off)
    lens_pin = pin(lens_pg.copy())
    for name, arr in (("pageable", lens_pg), ("pinned", lens_pin)):
        t0 = time.perf_counter()
        for _ in range(5):
            np.cumsum(arr, dtype=np.uint64)
        res[f"cumsum_{name}_ms"] = round((time.perf_counter() - t0) / 5 * 1e3, 3)
    epool2 = bench.PinnedPool()
    for name, al in (("encode_len_pageable", None), ("encode_len_pinned", epool2)):
        ts = []
        for _ in range(3):
            epool2.rewind()
            t0 = time.perf_counter()
            codec.encode_len(data, off, alloc=al) if al is not None else codec.encode_len(data, off)
            ts.append(round(b.nbytes / (time.perf_counter() - t0) / (1 << 30), 2))
        res[name + "_gib_s"] = ts
    for step in args.steps.split(","):
        t0 = time.perf_counter()
        if step == "devalloc":
            x = torch.empty(8 << 30, dtype=torch.uint8, device="cuda")
            x.fill_(1)
            torch.cuda.synchronize()
            del x
            torch.cuda.empty_cache()
        elif step == "devkeep":
            x = torch.empty(8 << 30, dtype=torch.uint8, device="cuda")
            x.fill_(1)
            torch.cuda.synchronize()
            del x
        elif step == "smallfree":
            x = torch.empty(64 << 20, dtype=torch.uint8, device="cuda")
            torch.cuda.synchronize()
            del x
            torch.cuda.empty_cache()
        elif step == "pageable":  # (not a disturbance: the decode rate into pageable outputs, for comparison)
            t0p = time.perf_counter()
            codec.decode(np.array(enc), np.array(eoff), np.array(cap))
            res["pageable_gib_s"] = round(b.nbytes / (time.perf_counter() - t0p) / (1 << 30), 2)
        elif step == "repin":  # inputs and output pool pinned afresh
            S.update(dpool=bench.PinnedPool(), enc=pin(np.array(enc)), eoff=pin(np.array(eoff)), cap=pin(np.array(cap)))
        elif step == "sleep":
            time.sleep(2)
        elif step == "pinalloc":
            x = torch.empty(2 << 30, dtype=torch.uint8).pin_memory()
            x.fill_(1)
            del x
        elif step == "bigdec":
            c5 = workloads.make_batch(4 << 20, "fixed", "adv", workloads.SEED_ADV, 128, 128)
            e5, o5 = codec.encode(c5.data, c5.off)
            codec.decode(e5, o5)
            del c5, e5, o5
        elif step == "lenbig":
            codec.encode_len(data, off)
        elif step == "encode":
            epool.rewind()
            codec.encode(data, off, alloc=epool)
        elif step == "newctx":
            with hc.Codec(devices=[0]) as c2:
                c2.decode(enc, eoff, cap)
        else:
            raise SystemExit(f"unknown step {step}")
        took = round(time.perf_counter() - t0, 2)
        res[step] = {"after": [dec() for _ in range(int(os.environ.get("HOSTPATH_AFTER", "3")))], "step_s": took,
                     "rawbw": rawbw()}
        print(step, res[step], file=sys.stderr, flush=True)
    res["env"] = {k: os.environ.get(k) for k in ("MHQ_HOST_CHUNK_MB", "MHQ_HOST_LEN_CHUNK_MB")}
    print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()
