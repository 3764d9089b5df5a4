#!/usr/bin/env python3
"""A/B of read_strings across builds of libmhq_huff.so, in one process.

    python tools/ab_read.py --libs base=minhq_amd/libmhq_huff.so,fused=build/v/lib_fused.so

Cases: `hdr` (tools/bench_rows.py's block: config-2 literals, Huffman, 7-bit
prefix), `mixed` (Auto choice -- raw and Huffman --, prefixes 1..7, opcode
bits), `zipf` (long literals: tiles that stream), `shuffled` (pos out of block
order: the scan layout), `long` (300-600 B literals: every tile streams), `garbage` (random bytes as frames).  Every library's
out_off / out_len / status / next and the bytes inside each string's length
must equal base's; the first prints the median us per call of each library.
"""
from __future__ import annotations

import argparse
import ctypes as C
import json
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))

from abmulti import open_lib  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--libs", required=True)
    ap.add_argument("--cases", default="hdr,mixed,zipf,long,shuffled,garbage")
    ap.add_argument("--n", type=int, default=1 << 20)
    ap.add_argument("--reps", type=int, default=3)
    ap.add_argument("--iters", type=int, default=20)
    ap.add_argument("--json", default="")
    args = ap.parse_args()

    import torch

    from minhq_amd import hc, workloads

    dev = torch.device("cuda:0")
    codec = hc.Codec(devices=[0])
    libs = []
    for item in args.libs.split(","):
        name, path = item.split("=", 1)
        libs.append((name,) + open_lib(path))
    stream = C.c_void_p(torch.cuda.current_stream().cuda_stream)
    rng = np.random.default_rng(11)
    results, ok = [], True
    for case in args.cases.split(","):
        n = args.n if case in ("hdr", "mixed") else args.n // 8
        if case == "zipf":
            b = workloads.make_batch(n, "zipf", "hdr")
        elif case == "long":
            b = workloads.make_batch(n // 8, "uniform", "hdr", lo=300, hi=600)
            n = n // 8
        else:
            b = workloads.make_batch(n, "uniform", "hdr", lo=0 if case == "mixed" else 8, hi=64)
        lits = hc.unpack(b.data, b.off)
        if case == "mixed":
            pfs = [int(x) for x in rng.integers(1, 8, size=n)]
            leads = [int(rng.integers(0, 1 << (7 - p))) for p in pfs]
            frames = codec.write_strings(lits, pfs, leads, hc.HuffmanCodingAuto)
        else:
            pfs = [7] * n
            frames = codec.write_strings(lits, pfs, None, hc.HuffmanCodingAlways)
        blk = np.frombuffer(b"".join(frames), dtype=np.uint8).copy()
        lens = np.array([len(f) for f in frames], dtype=np.uint64)
        pos = np.zeros(n, dtype=np.uint64)
        pos[1:] = np.cumsum(lens)[:-1]
        lim = np.full(n, len(blk), dtype=np.uint64)
        if case == "shuffled":
            perm = rng.permutation(n)
            pos = pos[perm]
            pfs = [pfs[i] for i in perm]
        if case == "garbage":
            blk = rng.integers(0, 256, size=len(blk), dtype=np.uint8)
            lim = np.minimum(pos + rng.integers(0, 80, size=n).astype(np.uint64), len(blk)).astype(np.uint64)
        t_blk = torch.from_numpy(blk).to(dev)
        t_pos = torch.from_numpy(pos.view(np.int64)).to(dev)
        t_lim = torch.from_numpy(lim.view(np.int64)).to(dev)
        t_pf = torch.tensor(pfs, dtype=torch.uint8, device=dev)
        cap = len(blk) * 8 // 5 + 16
        if case == "shuffled":
            cap = int(len(blk) * 8 // 5 + 16)
        outs = {}
        times = {name: [] for name, *_ in libs}
        for rep in range(args.reps):
            for name, L, h in libs:
                o = {"out": torch.zeros(cap, dtype=torch.uint8, device=dev),
                     "off": torch.empty(n + 1, dtype=torch.int64, device=dev),
                     "len": torch.empty(n, dtype=torch.int32, device=dev),
                     "st": torch.empty(n, dtype=torch.uint8, device=dev),
                     "nx": torch.empty(n, dtype=torch.int64, device=dev)}

                def run():
                    rc = L.mhq_read_strings_dev(h, 0, t_blk.data_ptr(), len(blk), t_pos.data_ptr(), t_lim.data_ptr(),
                                                t_pf.data_ptr(), n, o["out"].data_ptr(), cap, o["off"].data_ptr(),
                                                o["len"].data_ptr(), o["st"].data_ptr(), o["nx"].data_ptr(), stream)
                    if rc != 0:
                        raise RuntimeError(f"{name}: rc={rc}")

                for _ in range(3):
                    run()
                torch.cuda.synchronize()
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record()
                for _ in range(args.iters):
                    run()
                e1.record()
                torch.cuda.synchronize()
                times[name].append(e0.elapsed_time(e1) / args.iters * 1e3)
                if rep == 0:
                    outs[name] = o
        base = outs[libs[0][0]]
        ln = base["len"].long()
        idx = torch.repeat_interleave(base["off"][:-1], ln) + (
            torch.arange(int(ln.sum().item()), device=dev) - torch.repeat_interleave(torch.cumsum(ln, 0) - ln, ln))
        for name, *_ in libs[1:]:
            o = outs[name]
            diffs = [k for k in ("off", "len", "st", "nx") if not torch.equal(base[k], o[k])]
            if not diffs and not torch.equal(base["out"][idx], o["out"][idx]):
                diffs.append("bytes")
            print(f"check {case} {name}: {'SAME' if not diffs else 'DIFFERENT ' + ','.join(diffs)}", flush=True)
            ok = ok and not diffs
        for name, *_ in libs:
            t = np.array(times[name])
            r = {"case": case, "lib": name, "n": n, "us_med": round(float(np.median(t)), 2),
                 "us_min": round(float(t.min()), 2), "all": [round(x, 2) for x in t]}
            results.append(r)
            print(f"{case:9s} {name:10s} n={n:8d} med {r['us_med']:8.2f} min {r['us_min']:8.2f} us {r['all']}",
                  flush=True)
        del outs
        torch.cuda.empty_cache()
    if args.json:
        with open(args.json, "w") as f:
            json.dump(results, f, indent=1)
    codec.close()
    sys.exit(0 if ok else 1)


if __name__ == "__main__":
    main()
