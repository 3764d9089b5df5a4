#!/usr/bin/env python3
"""Minimal driver for profiling one kernel of libmhq_huff.so.

    python tools/kernel_driver.py --kernel decode --config northstar --iters 50

Prepares the batch on the device (encoding it first for decode), then times
`--iters` launches over rotating buffer copies (>= 1 GiB) with HIP events, and
prints one JSON line.  Meant to run under `rocprofv3 --kernel-trace` or
`--pmc`; MHQ_LIB_PATH may point at a variant build.
"""
from __future__ import annotations

import argparse
import json
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def batch_for(name: str, n: int):
    from minhq_amd import workloads as w

    if name == "northstar":
        return w.north_star(n or (1 << 20))
    if name == "config2":
        return w.config2(n or (1 << 20))
    if name == "config2print":
        return w.config2(n or (1 << 20), "print")
    if name == "config3":  # the QIF corpus: netbsd.qif's literals (+ test texts) tiled to 2^20
        return w.config3(n or (1 << 20))
    if name == "config4":
        return w.config4(n or (1 << 22))
    if name == "config5":
        return w.config5(n or (1 << 20))
    if ":" in name:  # kind:lo:hi, e.g. uniform:8:96 or zipf:4:256 (hdr bytes, 2^20 literals)
        kind, lo, hi = name.split(":")
        return w.make_batch(n or (1 << 20), kind, "hdr", 12345, int(lo), int(hi), name)
    raise SystemExit(f"unknown config {name}")


def timeline_report(fn):
    """Summarises the MHQ_DIAG_TIMELINE build's per-wave stamps (last launch):
    slot 0 start, 63 end, tile j: 1+5j+k, k = 0 next loads issued, 1 previous
    output flushed, 2 sorted, 3 fast loop done, 4 decoded."""
    import ctypes

    W, S = 1024 * 16, 64
    buf = (ctypes.c_ulonglong * (W * S))()
    fn(buf, W * S)
    a = np.frombuffer(buf, dtype=np.uint64).reshape(W, S).astype(np.int64)
    wave_id = np.nonzero(a[:, 0] > 0)[0]
    a = a[a[:, 0] > 0]
    t0 = a[:, 0].min()
    us = lambda x: (x - t0) / 100.0  # 100 MHz ticks -> us
    end = us(a[:, S - 1])
    blk = wave_id // 16
    blk_end = {}
    for b_, e_ in zip(blk, end):
        blk_end[b_] = max(blk_end.get(b_, 0.0), e_)
    be = np.array([blk_end[b_] for b_ in sorted(blk_end)])
    bx = np.array(sorted(blk_end)) % 8
    print("  workgroup end by XCD (blockIdx % 8): " + " ".join(
        f"{x}:{be[bx == x].mean():.1f}/{be[bx == x].max():.1f}" for x in range(8)) +
        f"  | workgroup end p10 {np.percentile(be, 10):.1f} p50 {np.percentile(be, 50):.1f} max {be.max():.1f}",
        file=sys.stderr)
    wix = wave_id % 16
    print("  wave end by wave index (mean): " + " ".join(
        f"{w}:{end[wix == w].mean():.1f}" for w in range(16) if (wix == w).any()), file=sys.stderr)
    for j in range(3):
        b = 1 + 5 * j
        cols = []
        for g in range(4):
            sel = (wix // 4 == g) & (a[:, b + 4] > 0)
            if sel.any():
                x = a[sel]
                cols.append(f"g{g}: issued@{us(x[:, b]).mean():.1f} sorted@{us(x[:, b + 2]).mean():.1f} "
                            f"loop {(x[:, b + 3] - x[:, b + 2]).mean() / 100:.2f} done@{us(x[:, b + 4]).mean():.1f}")
        print(f"  tile {j} by age group: " + " | ".join(cols), file=sys.stderr)
    for slot, what in ((56, "first offsets in"), (57, "tables in LDS"), (58, "first input staged")):
        ok = a[:, slot] > 0
        if ok.any():
            print(f"  opening: {what} @{us(a[ok, slot]).mean():.2f} us (p90 {np.percentile(us(a[ok, slot]), 90):.2f})",
                  file=sys.stderr)
    print(f"timeline: {a.shape[0]} waves, start spread {us(a[:, 0]).max():.2f} us, end max {end.max():.2f} "
          f"p50 {np.percentile(end, 50):.2f} p10 {np.percentile(end, 10):.2f} us", file=sys.stderr)
    prev = a[:, 0]
    for j in range(12):
        b = 1 + 5 * j
        ok = a[:, b + 4] > 0
        if not ok.any():
            break
        x = a[ok]
        pv = prev[ok]
        d = lambda k0, k1: (x[:, b + k1] - x[:, b + k0]).mean() / 100
        print(f"  tile {j}: waves={ok.sum()} stage {(x[:, b] - pv).mean() / 100:.2f} flush {d(0, 1):.2f} "
              f"sort {d(1, 2):.2f} fast {d(2, 3):.2f} tails {d(3, 4):.2f} "
              f"(decode p90 {np.percentile(x[:, b + 4] - x[:, b + 1], 90) / 100:.2f}) "
              f"done@{us(x[:, b + 4]).mean():.2f}", file=sys.stderr)
        prev = np.where(a[:, b + 4] > 0, a[:, b + 4], prev)


def etimeline_report(fn):
    """Summarises the MHQ_DIAG_ETL build's per-wave coop-encode stamps (last
    launch): [0] start, [1] table ready, [2] offsets used, [3] first loads
    issued, [4 + r] round r done, [63] end."""
    import ctypes

    W, S = 16384, 64
    buf = (ctypes.c_ulonglong * (W * S))()
    fn(buf, W * S)
    a = np.frombuffer(buf, dtype=np.uint64).reshape(W, S).astype(np.int64)
    a = a[(a[:, 0] > 0) & (a[:, 63] > 0)]
    t0 = a[:, 0].min()
    us = lambda x: (x - t0) / 100.0  # noqa: E731
    st = us(a[:, 0])
    print(f"etl: {a.shape[0]} waves; start p10 {np.percentile(st, 10):.2f} p50 {np.percentile(st, 50):.2f} "
          f"p90 {np.percentile(st, 90):.2f} max {st.max():.2f}; end p50 {np.percentile(us(a[:, 63]), 50):.2f} "
          f"max {us(a[:, 63]).max():.2f} us", file=sys.stderr)
    d = lambda k0, k1: (a[:, k1] - a[:, k0]) / 100.0  # noqa: E731
    print(f"  per wave (mean us): table {d(0, 1).mean():.2f} offsets {d(1, 2).mean():.2f} issue {d(2, 3).mean():.2f} "
          f"round0 {d(3, 4).mean():.2f} life {d(0, 63).mean():.2f}", file=sys.stderr)
    nr = (a[:, 4:62] > 0).sum(axis=1)
    rounds = []
    for r in range(1, 12):
        ok = nr > r
        if ok.sum() < 10:
            break
        rounds.append(f"r{r} {((a[ok, 4 + r] - a[ok, 3 + r]) / 100.0).mean():.2f}")
    last = a[np.arange(a.shape[0]), 3 + nr]
    print(f"  rounds per wave mean {nr.mean():.2f}; round durations: " + " ".join(rounds) +
          f"; tail (last round -> end) {((a[:, 63] - last) / 100.0).mean():.2f}", file=sys.stderr)
    # by start generation
    gen = np.digitize(st, np.percentile(st, [25, 50, 75]))
    print("  by start quartile: " + " | ".join(
        f"q{g}: start {st[gen == g].mean():.1f} life {d(0, 63)[gen == g].mean():.2f} "
        f"round0 {d(3, 4)[gen == g].mean():.2f}" for g in range(4) if (gen == g).any()), file=sys.stderr)


def pktimeline_report(fn, nwg):
    """Summarises the MHQ_DIAG_PKTL build's per-workgroup stamps of the packed
    encode (last launch): [0] start, [1] staged, [2] sorted, [3] sized, [4]
    scanned + published, [5] wave 0 encoded, [6] look-back done, [7] base
    barrier, [8] end."""
    import ctypes

    W, S = 8192, 16
    buf = (ctypes.c_ulonglong * (W * S))()
    fn(buf, W * S)
    a = np.frombuffer(buf, dtype=np.uint64).reshape(W, S).astype(np.int64)[:nwg]
    a = a[(a[:, 0] > 0) & (a[:, 8] > 0)]
    t0 = a[:, 0].min()
    st = (a[:, 0] - t0) / 100.0
    end = (a[:, 8] - t0) / 100.0
    print(f"pktl: {a.shape[0]} workgroups; start p25 {np.percentile(st, 25):.2f} p50 {np.percentile(st, 50):.2f} "
          f"p75 {np.percentile(st, 75):.2f} max {st.max():.2f}; end p50 {np.median(end):.2f} max {end.max():.2f} us",
          file=sys.stderr)
    d = lambda k0, k1: (a[:, k1] - a[:, k0]) / 100.0  # noqa: E731
    names = ["stage", "sort", "size", "scan+pub", "encode(w0)", "lookback", "barrier", "store"]
    print("  per workgroup (mean us): " + " ".join(f"{nm} {d(k, k + 1).mean():.2f}" for k, nm in enumerate(names)) +
          f" life {d(0, 8).mean():.2f}", file=sys.stderr)
    gen = np.digitize(st, np.percentile(st, [25, 50, 75]))
    print("  by start quartile: " + " | ".join(
        f"q{g}: start {st[gen == g].mean():.1f} life {d(0, 8)[gen == g].mean():.2f} lb {d(5, 6)[gen == g].mean():.2f}"
        for g in range(4) if (gen == g).any()), file=sys.stderr)
    # concurrency: resident workgroups over time
    tt = np.linspace(0, end.max(), 12)
    res = [int(((st <= x) & (end > x)).sum()) for x in tt]
    print("  resident over time: " + " ".join(f"{x:.1f}:{r}" for x, r in zip(tt, res)), file=sys.stderr)


def wg_report(fn):
    """Summarises the MHQ_DIAG_WG build's stamps (last launch): stager tile
    timeline and decoder wait/work split, in us from the workgroup's start."""
    import ctypes

    T, D = 4, 132
    S = D + 4 * 16
    buf = (ctypes.c_ulonglong * (1024 * S))()
    fn(buf, 1024 * S)
    a = np.frombuffer(buf, dtype=np.uint64).reshape(1024, S).astype(np.int64)
    a = a[a[:, 0] > 0]
    t0 = a[:, 0:1]
    us = lambda x: (x - t0) / 100.0  # noqa: E731
    print(f"wg: {a.shape[0]} workgroups, tiles/wg mean {a[:, 3].mean() + 1:.1f}; first publish "
          f"{np.median(us(a[:, 1:2])):.2f} us, stager end {np.median(us(a[:, 2:3])):.2f} us", file=sys.stderr)
    names = ["stage", "offsets", "published", "freed", "dma-issued", "records", "last-sub-done", "flush-issued"]
    for k in range(10):
        b = T + 8 * k
        ok = a[:, b] > 0
        if not ok.any():
            break
        x = a[ok]
        cols = []
        for q, nm in enumerate(names):
            v = x[:, b + q]
            good = v > 0
            cols.append(f"{nm}@{np.median((v[good] - x[good, 0]) / 100.0):.2f}" if good.any() else f"{nm}@-")
        print(f"  tile {k}: " + " ".join(cols), file=sys.stderr)
    dec = a[:, D:].reshape(a.shape[0], 16, 4)
    live = dec[:, :, 3] > 0
    wait = dec[:, :, 0][live] / 100.0
    work = dec[:, :, 1][live] / 100.0
    end = (dec[:, :, 3] - a[:, 0:1])[live] / 100.0
    print(f"  decoders: wait {wait.mean():.2f} us, decode {work.mean():.2f} us, sub-tiles "
          f"{dec[:, :, 2][live].mean():.2f}, end p50 {np.median(end):.2f} max {end.max():.2f} us", file=sys.stderr)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--kernel", default="decode", choices=["decode", "encode", "encode_len", "offsets", "layout", "packed"])
    ap.add_argument("--config", default="northstar")
    ap.add_argument("--n", type=int, default=0)
    ap.add_argument("--iters", type=int, default=50)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--rotate-gib", type=float, default=1.0)
    ap.add_argument("--no-check", action="store_true")
    ap.add_argument("--exact", action="store_true", help="decode into regions of the exact plaintext length")
    args = ap.parse_args()

    import torch

    from minhq_amd import hc

    b = batch_for(args.config, args.n)
    dev = torch.device("cuda:0")
    codec = hc.Codec(devices=[0])
    n = b.n
    data = torch.from_numpy(b.data).to(dev)
    off = torch.from_numpy(b.off.view(np.int64)).to(dev)
    enc_len = torch.empty(n, dtype=torch.int32, device=dev)
    enc_off = torch.empty(n + 1, dtype=torch.int64, device=dev)
    cap_off = torch.empty(n + 1, dtype=torch.int64, device=dev)
    codec.encode_len_dev(data, off, enc_len)
    codec.offsets_dev(enc_len, enc_off, cap_off)
    torch.cuda.synchronize()
    enc_bytes = int(enc_off[-1].item())
    cap_bytes = int(cap_off[-1].item())
    enc = torch.empty(enc_bytes + 16, dtype=torch.uint8, device=dev)
    codec.encode_dev(data, off, enc, enc_off)
    torch.cuda.synchronize()
    if args.exact:  # the plaintext offsets as the output layout (a round trip knows them)
        cap_off = off - off[0]
        cap_bytes = int(cap_off[-1].item())

    per = {"decode": enc_bytes + cap_bytes + 16 * n, "encode": b.nbytes + enc_bytes + 16 * n,
           "encode_len": b.nbytes + 12 * n, "offsets": 20 * n, "layout": b.nbytes + 32 * n,
           "packed": b.nbytes + enc_bytes + 28 * n}[args.kernel]
    R = max(2, int(np.ceil(args.rotate_gib * (1 << 30) / per)))
    slots = []
    for _ in range(R):
        s = {}
        if args.kernel == "decode":
            s["in"], s["off"], s["cap"] = enc.clone(), enc_off.clone(), cap_off.clone()
            s["out"] = torch.empty(cap_bytes + 16, dtype=torch.uint8, device=dev)
            s["len"] = torch.empty(n, dtype=torch.int32, device=dev)
            s["st"] = torch.empty(n, dtype=torch.uint8, device=dev)
        elif args.kernel in ("encode", "encode_len", "layout", "packed"):
            s["in"], s["off"], s["eoff"] = data.clone(), off.clone(), enc_off.clone()
            s["out"] = torch.empty(30 * b.nbytes // 8 + n if args.kernel == "packed" else enc_bytes + 16,
                                   dtype=torch.uint8, device=dev)
            s["len"] = torch.empty(n, dtype=torch.int32, device=dev)
            s["o1"] = torch.empty_like(enc_off)
            s["o2"] = torch.empty_like(cap_off)
        else:
            s["len"] = enc_len.clone()
            s["o1"] = torch.empty_like(enc_off)
            s["o2"] = torch.empty_like(cap_off)
        slots.append(s)

    def run(s):
        if args.kernel == "decode":
            codec.decode_dev(s["in"], s["off"], s["out"], s["cap"], s["len"], s["st"])
        elif args.kernel == "encode":
            codec.encode_dev(s["in"], s["off"], s["out"], s["eoff"])
        elif args.kernel == "encode_len":
            codec.encode_len_dev(s["in"], s["off"], s["len"])
        elif args.kernel == "layout":
            codec.encode_layout_dev(s["in"], s["off"], s["len"], s["o1"], s["o2"])
        elif args.kernel == "packed":
            codec.encode_packed_dev(s["in"], s["off"], b.nbytes, s["len"], s["o1"], s["o2"], s["out"])
        else:
            codec.offsets_dev(s["len"], s["o1"], s["o2"])

    for i in range(args.warmup):
        run(slots[i % R])
    torch.cuda.synchronize()
    import ctypes

    from minhq_amd import _lib

    diag = getattr(_lib.load(), "mhq_diag_read", None)
    buf = (ctypes.c_ulonglong * 8)()
    if diag:
        diag(buf, 8)  # reset
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for i in range(args.iters):
        run(slots[i % R])
    e1.record()
    torch.cuda.synchronize()
    ms = e0.elapsed_time(e1) / args.iters
    if diag:
        diag(buf, 8)
        it, lanes = buf[0] / args.iters, buf[1] / args.iters
        print(f"diag counts per launch: fast-loop wave iterations {it:.4g}, active lanes {lanes:.4g} "
              f"(utilisation {lanes / max(it * 64, 1):.3f}), per literal {lanes / n:.2f} lane-steps", file=sys.stderr)
    wg = getattr(_lib.load(), "mhq_diag_wg", None)
    if wg:
        wg_report(wg)
    etl = getattr(_lib.load(), "mhq_diag_etimeline", None)
    if etl:
        etimeline_report(etl)
    pk = getattr(_lib.load(), "mhq_diag_pktimeline", None)
    if pk and args.kernel == "packed":
        pktimeline_report(pk, min(8192, (n + 255) // 256))
    tl = getattr(_lib.load(), "mhq_diag_timeline", None)
    if tl:
        timeline_report(tl)
    if args.kernel == "decode" and not args.no_check:
        s = slots[0]
        assert int(s["st"].sum().item()) == 0
        assert torch.equal(s["len"].long(), off[1:] - off[:-1])
    alg = {"decode": enc_bytes + b.nbytes + 16 * (n + 1) + 5 * n,
           "encode": b.nbytes + enc_bytes + 16 * (n + 1) + 4 * n,  # + 4n (enc_len)
           "encode_len": b.nbytes + 8 * (n + 1) + 4 * n, "offsets": 4 * n + 16 * (n + 1),
           "layout": b.nbytes + 8 * (n + 1) + 8 * n + 16 * (n + 1),
           "packed": b.nbytes + enc_bytes + 8 * (n + 1) + 4 * n + 16 * (n + 1)}[args.kernel]
    print(json.dumps({"kernel": args.kernel, "config": b.name, "n": n, "plain": b.nbytes, "enc": enc_bytes,
                      "us_per_launch": round(ms * 1e3, 2), "plain_gib_s": round(b.nbytes / ms / 1e6 / 1.073741824, 2),
                      "alg_bytes": alg, "hbm_frac": round(alg / (ms / 1e3) / 8e12, 4), "rotating": R}))


if __name__ == "__main__":
    main()
