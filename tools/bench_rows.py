#!/usr/bin/env python3
"""Measurements for the §8(f) rows beside the headline path (GPU box):

  * read_strings_dev: batch Reader.ReadString over one block of framed
    literals (H bit + 7-bit prefix + payload), device-resident, GiB/s of
    decoded output; the parse, scans, gather, decode and finish kernels all
    inside the timed region;
  * read_ints_dev: batch Reader.ReadInt, integers/s;
  * read_varints_dev: batch frameReader.ReadVarint, varints/s;
  * HPACK batch header-block decode (minhq_amd.headers): host walk, GPU
    string batch and table replay timed separately, beside the same blocks
    through the CPU oracle's ReadString (one core).

Prints one JSON line.  python3 tools/bench_rows.py [--literals N]
"""
import argparse
import json
import os
import random
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)

import numpy as np  # noqa: E402
import torch  # noqa: E402

from minhq_amd import hc, workloads  # noqa: E402
from minhq_amd.headers import HpackBatchDecoder  # noqa: E402
from oracle import oracle  # noqa: E402


def timed(fn, iters, warm=3):
    for _ in range(warm):
        fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(iters):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / iters  # ms


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--literals", type=int, default=1 << 20)
    ap.add_argument("--blocks", type=int, default=20000)
    args = ap.parse_args()
    dev = torch.device("cuda:0")
    codec = hc.Codec(devices=[0])
    oracle.build()
    res = {}

    # framed string literals: the config-2 batch, each literal Huffman-framed by the GPU writer
    b = workloads.make_batch(args.literals, "uniform", "hdr", lo=8, hi=64)
    lits = hc.unpack(b.data, b.off)
    frames = codec.write_strings(lits, [7] * len(lits), None, hc.HuffmanCodingAlways)
    blk = np.frombuffer(b"".join(frames), dtype=np.uint8)
    lens = np.array([len(f) for f in frames], dtype=np.uint64)
    pos = np.zeros(len(frames), dtype=np.uint64)
    pos[1:] = np.cumsum(lens)[:-1]
    t_blk = torch.from_numpy(blk.copy()).to(dev)
    t_pos = torch.from_numpy(pos.view(np.int64)).to(dev)
    t_lim = torch.full((len(frames),), len(blk), dtype=torch.int64, device=dev)
    t_pf = torch.full((len(frames),), 7, dtype=torch.uint8, device=dev)
    n = len(frames)
    out = torch.empty(len(blk) * 8 // 5 + 16, dtype=torch.uint8, device=dev)
    out_off = torch.empty(n + 1, dtype=torch.int64, device=dev)
    out_len = torch.empty(n, dtype=torch.int32, device=dev)
    st = torch.empty(n, dtype=torch.uint8, device=dev)
    nxt = torch.empty(n, dtype=torch.int64, device=dev)
    ms = timed(lambda: codec.read_strings_dev(t_blk, t_pos, t_lim, t_pf, out, out_off, out_len, st, nxt), 10)
    assert int(out_len.sum().item()) == b.nbytes and int((st != 0).sum().item()) == 0
    # the bare decode of the same literals (packed encodings, floor(8C/5) regions)
    d_data = torch.from_numpy(b.data).to(dev)
    d_off = torch.from_numpy(b.off.view(np.int64)).to(dev)
    e_len = torch.empty(n, dtype=torch.int32, device=dev)
    e_off = torch.empty(n + 1, dtype=torch.int64, device=dev)
    c_off = torch.empty(n + 1, dtype=torch.int64, device=dev)
    codec.encode_layout_dev(d_data, d_off, e_len, e_off, c_off)
    torch.cuda.synchronize()
    enc = torch.empty(int(e_off[-1].item()) + 16, dtype=torch.uint8, device=dev)
    codec.encode_dev(d_data, d_off, enc, e_off)
    dout = torch.empty(int(c_off[-1].item()) + 16, dtype=torch.uint8, device=dev)
    bare = timed(lambda: codec.decode_dev(enc, e_off, dout, c_off, out_len, st), 10)
    assert int(out_len.sum().item()) == b.nbytes and int((st != 0).sum().item()) == 0
    res["read_strings_dev"] = {"strings": n, "block_bytes": int(len(blk)), "decoded_bytes": int(b.nbytes),
                               "ms": round(ms, 4), "decoded_gib_s": round(b.nbytes / (ms * 1e-3) / 2**30, 2),
                               "bare_decode_ms": round(bare, 4), "ratio_to_bare_decode": round(ms / bare, 3)}

    # prefix integers: random values / prefixes framed by the GPU writer
    rng = np.random.default_rng(7)
    vals = rng.integers(0, 1 << 20, size=args.literals, dtype=np.uint64)
    pfs = rng.integers(3, 9, size=args.literals).astype(np.uint8)
    ints = codec.write_ints([int(v) for v in vals], pfs)
    iblk = np.frombuffer(b"".join(ints), dtype=np.uint8)
    ipos = np.zeros(len(ints), dtype=np.uint64)
    ipos[1:] = np.cumsum([len(x) for x in ints])[:-1]
    t_iblk = torch.from_numpy(iblk.copy()).to(dev)
    t_ipos = torch.from_numpy(ipos.view(np.int64)).to(dev)
    t_ilim = torch.full((len(ints),), len(iblk), dtype=torch.int64, device=dev)
    t_ipf = torch.from_numpy(pfs).to(dev)
    t_val = torch.empty(len(ints), dtype=torch.int64, device=dev)
    t_inx = torch.empty(len(ints), dtype=torch.int64, device=dev)
    t_ist = torch.empty(len(ints), dtype=torch.uint8, device=dev)
    ms = timed(lambda: codec.read_ints_dev(t_iblk, t_ipos, t_ilim, t_ipf, t_val, t_inx, t_ist), 20)
    assert np.array_equal(t_val.cpu().numpy().view(np.uint64), vals)
    res["read_ints_dev"] = {"ints": len(ints), "ms": round(ms, 4), "gints_s": round(len(ints) / (ms * 1e-3) / 1e9, 2)}

    # HTTP/3 (draft) varints of every length class
    vv = rng.integers(0, 1 << 62, size=args.literals, dtype=np.uint64) >> rng.integers(
        0, 62, size=args.literals).astype(np.uint64)
    encs, _ = codec.write_varints([int(v) for v in vv])
    vblk = np.frombuffer(b"".join(encs), dtype=np.uint8)
    vpos = np.zeros(len(encs), dtype=np.uint64)
    vpos[1:] = np.cumsum([len(x) for x in encs])[:-1]
    t_vblk = torch.from_numpy(vblk.copy()).to(dev)
    t_vpos = torch.from_numpy(vpos.view(np.int64)).to(dev)
    t_vlim = torch.full((len(encs),), len(vblk), dtype=torch.int64, device=dev)
    t_vval = torch.empty(len(encs), dtype=torch.int64, device=dev)
    t_vnx = torch.empty(len(encs), dtype=torch.int64, device=dev)
    t_vst = torch.empty(len(encs), dtype=torch.uint8, device=dev)
    ms = timed(lambda: codec.read_varints_dev(t_vblk, t_vpos, t_vlim, t_vval, t_vnx, t_vst), 20)
    assert np.array_equal(t_vval.cpu().numpy().view(np.uint64), vv)
    res["read_varints_dev"] = {"varints": len(encs), "ms": round(ms, 4),
                               "gvarints_s": round(len(encs) / (ms * 1e-3) / 1e9, 2)}

    # HPACK blocks of literals (Huffman by Auto) from the netbsd.qif header set
    with open(os.path.join(REPO, "tests", "golden", "netbsd_qif.json")) as f:
        fields = [(x[0].encode(), x[1].encode()) for x in json.load(f)["fields"] if x]
    r = random.Random(1)
    blocks = []
    for _ in range(args.blocks):
        hs = [fields[r.randrange(len(fields))] for _ in range(r.randint(4, 16))]
        hs.sort(key=lambda h: not h[0].startswith(b":"))
        blocks.append(b"".join(bytes([0]) + oracle.write_string(a, 7) + oracle.write_string(v, 7) for a, v in hs))
    dec = HpackBatchDecoder()
    dec.read_header_blocks(blocks[:100])
    t0 = time.perf_counter()
    got = dec.read_header_blocks(blocks)
    t1 = time.perf_counter()
    nfields = sum(len(x) for x in got)

    def oracle_reader(blk, pos, prefix, limit):
        vs, sts, nx = [], [], []
        for p, pf, lim in zip(pos, prefix, limit):
            v, rc, used = oracle.read_string(blk[p:lim], pf, skip_bits=7 - pf)
            vs.append(v)
            sts.append(0 if rc == 0 else 1)
            nx.append(p + used)
        return vs, sts, nx

    t2 = time.perf_counter()
    got_cpu = HpackBatchDecoder(oracle_reader).read_header_blocks(blocks)
    t3 = time.perf_counter()
    assert got_cpu == got
    res["hpack_batch"] = {"blocks": len(blocks), "fields": nfields, "wall_s": round(t1 - t0, 3),
                          "fields_per_s": round(nfields / (t1 - t0)), "cpu_oracle_reader_wall_s": round(t3 - t2, 3),
                          "note": "host walk + replay in Python; string literals in one mhq_read_strings call"}
    print(json.dumps(res), flush=True)
    codec.close()


if __name__ == "__main__":
    main()
