#!/usr/bin/env python3
"""A/B timing of several builds of libmhq_huff.so in ONE process.

    python tools/abmulti.py --kernel decode --configs northstar,config3 \
        --libs base=minhq_amd/libmhq_huff.so,nodec=build/v/lib_nodec.so --reps 3

Each config's batch is prepared once (with the in-tree library); every
library is loaded side by side (ctypes, RTLD_LOCAL) with its own context, and
the libraries are timed interleaved, `--reps` rounds, over rotating buffer
copies (>= --rotate-gib), HIP events on the current stream.  Prints one line
per (config, lib): median and min us per launch and the HBM fraction of the
median.  Timing builds (tools/abvar.sh) may produce wrong output; nothing is
checked unless --check names the libraries whose output must equal base's.
"""
from __future__ import annotations

import argparse
import ctypes as C
import json
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def open_lib(path):
    from minhq_amd import _lib

    L = C.CDLL(os.path.abspath(path))
    for name, (res, args) in _lib.SIGNATURES.items():
        fn = getattr(L, name, None)
        if fn is not None:
            fn.restype = res
            fn.argtypes = args
    h = C.c_void_p()
    dev = (C.c_int * 1)(0)
    rc = L.mhq_open_devices(C.byref(h), dev, 1)
    if rc != 0:
        raise RuntimeError(f"mhq_open_devices({path}) rc={rc}")
    return L, h


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--kernel", default="decode", choices=["decode", "encode", "layout", "packed", "layenc"])
    ap.add_argument("--configs", default="northstar")
    ap.add_argument("--libs", required=True)
    ap.add_argument("--reps", type=int, default=3)
    ap.add_argument("--iters", type=int, default=20)
    ap.add_argument("--rotate-gib", type=float, default=1.0)
    ap.add_argument("--check", default="", help="libs whose decode output must equal base's")
    ap.add_argument("--exact", action="store_true")
    ap.add_argument("--sized", action="store_true", help="decode through mhq_huff_decode_sized_dev (the batch's encoded bytes given)")
    ap.add_argument("--json", default="")
    args = ap.parse_args()

    import torch

    from minhq_amd import hc
    from kernel_driver import batch_for  # noqa: E402  (tools/ on sys.path)

    libs = []
    for item in args.libs.split(","):
        name, path = item.split("=", 1)
        libs.append((name, path) + open_lib(path))
    dev = torch.device("cuda:0")
    codec = hc.Codec(devices=[0])
    stream = C.c_void_p(torch.cuda.current_stream().cuda_stream)
    results = []
    for cfg in args.configs.split(","):
        b = batch_for(cfg, 0)
        n = b.n
        data = torch.from_numpy(b.data).to(dev)
        off = torch.from_numpy(b.off.view(np.int64)).to(dev)
        enc_len = torch.empty(n, dtype=torch.int32, device=dev)
        enc_off = torch.empty(n + 1, dtype=torch.int64, device=dev)
        cap_off = torch.empty(n + 1, dtype=torch.int64, device=dev)
        codec.encode_layout_dev(data, off, enc_len, enc_off, cap_off)
        torch.cuda.synchronize()
        enc_bytes = int(enc_off[-1].item())
        enc = torch.empty(enc_bytes + 16, dtype=torch.uint8, device=dev)
        codec.encode_dev(data, off, enc, enc_off)
        torch.cuda.synchronize()
        if args.exact:
            cap_off = off - off[0]
        cap_bytes = int(cap_off[-1].item())
        if args.kernel == "decode":
            per = enc_bytes + cap_bytes + 16 * n
            alg = enc_bytes + b.nbytes + 16 * (n + 1) + 5 * n
        elif args.kernel == "encode":
            per = b.nbytes + enc_bytes + 16 * n
            alg = b.nbytes + enc_bytes + 16 * (n + 1) + 4 * n
        elif args.kernel in ("packed", "layenc"):  # the encode side: plaintext in, lengths, offsets, codes out
            per = b.nbytes + 30 * b.nbytes // 8 + 33 * n
            alg = b.nbytes + enc_bytes + 8 * (n + 1) + 4 * n + 8 * (n + 1) + 8 * (n + 1)
        else:
            per = b.nbytes + 32 * n
            alg = b.nbytes + 8 * (n + 1) + 8 * n + 16 * (n + 1)
        R = max(2, int(np.ceil(args.rotate_gib * (1 << 30) / per)))
        slots = []
        for _ in range(R):
            s = {}
            if args.kernel == "decode":
                s["in"], s["off"], s["cap"] = enc.clone(), enc_off.clone(), cap_off.clone()
                s["out"] = torch.empty(cap_bytes + 16, dtype=torch.uint8, device=dev)
                s["len"] = torch.empty(n, dtype=torch.int32, device=dev)
                s["st"] = torch.empty(n, dtype=torch.uint8, device=dev)
            else:
                s["in"], s["off"] = data.clone(), off.clone()
                s["eoff"] = enc_off.clone()
                s["out"] = torch.empty(max(enc_bytes + 16, 30 * b.nbytes // 8 + n), dtype=torch.uint8, device=dev)
                s["len"] = torch.empty(n, dtype=torch.int32, device=dev)
                s["o1"] = torch.empty_like(enc_off)
                s["o2"] = torch.empty_like(cap_off)
            slots.append(s)

        def run(L, h, s):
            if args.kernel == "decode" and args.sized and hasattr(L, "mhq_huff_decode_sized_dev"):
                rc = L.mhq_huff_decode_sized_dev(h, 0, s["in"].data_ptr(), s["off"].data_ptr(), n, enc_bytes,
                                                 s["out"].data_ptr(), s["cap"].data_ptr(), s["len"].data_ptr(),
                                                 s["st"].data_ptr(), stream)
            elif args.kernel == "decode":
                rc = L.mhq_huff_decode_dev(h, 0, s["in"].data_ptr(), s["off"].data_ptr(), n, s["out"].data_ptr(),
                                           s["cap"].data_ptr(), s["len"].data_ptr(), s["st"].data_ptr(), stream)
            elif args.kernel == "encode":
                rc = L.mhq_huff_encode_dev(h, 0, s["in"].data_ptr(), s["off"].data_ptr(), n, s["out"].data_ptr(),
                                           s["eoff"].data_ptr(), stream)
            elif args.kernel == "packed":
                rc = L.mhq_huff_encode_packed_dev(h, 0, s["in"].data_ptr(), s["off"].data_ptr(), n, b.nbytes, 0,
                                                  s["len"].data_ptr(), s["o1"].data_ptr(), s["o2"].data_ptr(),
                                                  s["out"].data_ptr(), s["out"].numel(), stream)
            else:
                rc = L.mhq_huff_encode_layout_dev(h, 0, s["in"].data_ptr(), s["off"].data_ptr(), n, 0,
                                                  s["len"].data_ptr(), s["o1"].data_ptr(), s["o2"].data_ptr(),
                                                  stream)
                if rc == 0 and args.kernel == "layenc":
                    rc = L.mhq_huff_encode_dev(h, 0, s["in"].data_ptr(), s["off"].data_ptr(), n, s["out"].data_ptr(),
                                               s["o1"].data_ptr(), stream)
            if rc != 0:
                raise RuntimeError(f"rc={rc}")

        ref = None
        checks = set(x for x in args.check.split(",") if x)
        times = {name: [] for name, *_ in libs}
        for rep in range(args.reps):
            for name, path, L, h in libs:
                for i in range(3):
                    run(L, h, slots[i % R])
                torch.cuda.synchronize()
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record()
                for i in range(args.iters):
                    run(L, h, slots[i % R])
                e1.record()
                torch.cuda.synchronize()
                times[name].append(e0.elapsed_time(e1) / args.iters * 1e3)
                if rep == 0 and args.kernel == "decode" and (name == "base" or name in checks):
                    s = slots[(args.iters - 1) % R]
                    got = (s["out"].clone(), s["len"].clone(), s["st"].clone())
                    if name == "base":
                        ref = got
                    elif ref is not None:
                        same = all(torch.equal(a, c) for a, c in zip(ref[1:], got[1:]))
                        # bytes: compare only within each literal's decoded length
                        lens = ref[1].long()
                        o = s["cap"][:-1]
                        idx = torch.repeat_interleave(o, lens) + (
                            torch.arange(int(lens.sum().item()), device=dev) -
                            torch.repeat_interleave(torch.cumsum(lens, 0) - lens, lens))
                        same = same and torch.equal(ref[0][idx], got[0][idx])
                        print(f"check {cfg} {name}: {'SAME' if same else 'DIFFERENT'}", flush=True)
        for name, *_ in libs:
            t = np.array(times[name])
            r = {"config": cfg, "lib": name, "us_med": round(float(np.median(t)), 2), "us_min": round(float(t.min()), 2),
                 "hbm_frac": round(alg / (np.median(t) * 1e-6) / 8e12, 4), "all": [round(x, 2) for x in t]}
            results.append(r)
            print(f"{cfg:12s} {name:12s} med {r['us_med']:8.2f} min {r['us_min']:8.2f} us  frac {r['hbm_frac']:.4f}  "
                  f"{r['all']}", flush=True)
        del slots
        torch.cuda.empty_cache()
    if args.json:
        with open(args.json, "w") as f:
            json.dump(results, f, indent=1)


if __name__ == "__main__":
    main()
