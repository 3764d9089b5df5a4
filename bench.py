#!/usr/bin/env python3
"""bench.py -- device-resident Huffman literal GiB/s (encode+decode), 1..8 GPUs.

Metric (BASELINE.json): "device-resident Huffman literal GiB/s (encode+decode)".
Workload (BASELINE.json configs[1]): 2^20 synthetic header-field literals per
GPU, lengths U{8..64}, bytes drawn from the netbsd.qif header-byte histogram
(minhq_amd/workloads.py).  One step = one full round trip of
one batch on the device: encode_len -> offsets scan -> encode -> decode, all
through the C ABI (include/mhq_huff.h), inputs resident in HBM.  Rotating
copies of every buffer (>= 1 GiB in all) keep the 256 MB Infinity Cache from
serving a step's inputs from the previous step.

Consecutive batches alternate over 3 HIP streams (--streams; batches are
independent, a slot always runs on the same stream): one batch's first
kernels fill the CUs that the previous batch's decode leaves idle at its tail.

value = plaintext bytes of all ranks x steps / max-over-ranks wall time / 2^30.
Multi-GPU: one process per GPU (torchrun); each rank owns an independent shard
of literals (no data-path collective, weak scaling); the process group is used
only for the barrier and the max over ranks.

Extra fields (not `value`): the dominant kernel's roofline (decode), the
north-star decode-only rate (2^20 x U{8..56}), the PCIe-inclusive host-path
rate, and the CPU baseline (the oracle: minhq's Go algorithm restated in C,
oracle/huff_oracle.c; there is no Go toolchain on the box).
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

import numpy as np

REPO = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, REPO)

HBM_PEAK_GBS = 8000.0  # MI355X_MICROARCH.md: HBM3E 8.0 TB/s spec
GIB = float(1 << 30)


def log(*a):
    print(*a, file=sys.stderr, flush=True)


def dist_setup():
    import torch

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    torch.cuda.set_device(local)
    pg = None
    if world > 1:
        import torch.distributed as dist

        dist.init_process_group("nccl", device_id=torch.device("cuda", local))
        pg = dist
    return world, rank, local, pg


def barrier(pg):
    import torch

    torch.cuda.synchronize()
    if pg is not None:
        pg.barrier()
    torch.cuda.synchronize()


def max_over_ranks(pg, x: float) -> float:
    from minhq_amd import shard

    return shard.max_over_ranks(pg, x, "cuda")


class Slot:
    """One rotating copy of every buffer of a round-trip step."""

    def __init__(self, batch, enc_bytes, cap_bytes, dev):
        import torch

        n = batch.n
        self.n = n
        self.data = torch.from_numpy(batch.data).to(dev)
        self.off = torch.from_numpy(batch.off.view(np.int64)).to(dev)
        self.enc_len = torch.empty(n, dtype=torch.int32, device=dev)
        self.enc_off = torch.empty(n + 1, dtype=torch.int64, device=dev)
        self.cap_off = torch.empty(n + 1, dtype=torch.int64, device=dev)
        self.enc = torch.empty(enc_bytes + 16, dtype=torch.uint8, device=dev)
        self.out = torch.empty(cap_bytes + 16, dtype=torch.uint8, device=dev)
        self.out_len = torch.empty(n, dtype=torch.int32, device=dev)
        self.status = torch.empty(n, dtype=torch.uint8, device=dev)

    def nbytes(self):
        return sum(t.numel() * t.element_size() for t in
                   (self.data, self.off, self.enc_len, self.enc_off, self.cap_off, self.enc, self.out,
                    self.out_len, self.status))


def encoded_sizes(codec, batch, dev):
    import torch

    s = Slot(batch, 16, 16, dev)
    codec.encode_len_dev(s.data, s.off, s.enc_len)
    codec.offsets_dev(s.enc_len, s.enc_off, s.cap_off)
    torch.cuda.synchronize()
    return int(s.enc_off[-1].item()), int(s.cap_off[-1].item())


def round_trip(codec, s, stream=None):
    # encode_len + offsets scan (one call, two launches), encode, decode
    codec.encode_layout_dev(s.data, s.off, s.enc_len, s.enc_off, s.cap_off, stream=stream)
    codec.encode_dev(s.data, s.off, s.enc, s.enc_off, stream=stream)
    codec.decode_dev(s.enc, s.enc_off, s.out, s.cap_off, s.out_len, s.status, stream=stream)


def kernel_ms(codec, slots, which, launches):
    """Mean duration of one encode or decode launch over `launches`
    back-to-back launches rotating through the slots (HIP events on the
    current stream, which is the one the ABI calls launch on)."""
    import torch

    def run(s):
        if which == "encode":
            codec.encode_dev(s.data, s.off, s.enc, s.enc_off)
        else:
            codec.decode_dev(s.enc, s.enc_off, s.out, s.cap_off, s.out_len, s.status)

    for s in slots[:2]:
        run(s)
    stream = torch.cuda.current_stream()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record(stream)
    for i in range(launches):
        run(slots[i % len(slots)])
    e1.record(stream)
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / launches


def verify_slot(s, batch):
    import torch

    torch.cuda.synchronize()
    assert int(s.status.sum().item()) == 0, "decode reported INVALID on encoder output"
    assert torch.equal(s.out_len.long(), s.off[1:] - s.off[:-1]), "round trip length mismatch"


def decode_algorithmic_bytes(n, enc_bytes, plain_bytes):
    # sum C + sum out_len + 8(n+1) in_off + 8(n+1) out_off + 4n out_len + 1n status
    return enc_bytes + plain_bytes + 16 * (n + 1) + 5 * n


def load_traffic(path, kernel):
    try:
        with open(path) as f:
            d = json.load(f)
        return d.get(kernel, {}).get("hbm_bytes_per_launch")
    except Exception:
        return None


def cpu_baseline(batch, seconds: float):
    """The oracle (restated Go algorithm) on the host cores: encode + decode."""
    from minhq_amd import hc
    from oracle import oracle

    oracle.build()
    cores = max(1, min(16, os.cpu_count() or 1))
    m = min(batch.n, 1 << 17)
    off = batch.off[: m + 1].copy()
    data = batch.data[: int(off[-1])].copy()
    plain = int(off[-1])
    done = 0
    t0 = time.perf_counter()
    while True:
        enc_len = oracle.encode_len_batch(data, off, cores)
        eoff = np.zeros(m + 1, dtype=np.uint64)
        eoff[1:] = np.cumsum(enc_len, dtype=np.uint64)
        enc = oracle.encode_batch(data, off, eoff, cores)
        cap = hc.capacity_offsets(eoff)
        oracle.decode_batch(enc, eoff, cap, cores)
        done += 1
        el = time.perf_counter() - t0
        if el >= seconds:
            break
    return {"value": round(plain * done / el / GIB, 4), "unit": "GiB/s", "cores": cores, "kind": "port",
            "sample": f"first {m} literals of the workload, encode+decode x{done} passes in {el:.1f}s "
                      f"({cores} threads; minhq hc/huffman.go + io/bitio.go bit-serial algorithm "
                      f"restated in C, oracle/huff_oracle.c)"}


def decode_only(codec, dev, steps, warmup, rotate_bytes):
    """North-star decode-only rate: 2^20 x U{8..56} hdr literals."""
    import torch

    from minhq_amd import workloads

    b = workloads.north_star()
    enc_b, cap_b = encoded_sizes(codec, b, dev)
    base = Slot(b, enc_b, cap_b, dev)
    round_trip(codec, base)
    verify_slot(base, b)
    per = base.enc.numel() + base.enc_off.numel() * 16 + base.out.numel() + b.n * 5
    R = max(2, int(np.ceil(rotate_bytes / per)))
    slots = []
    for _ in range(R):
        s = type("S", (), {})()
        s.enc = base.enc.clone()
        s.enc_off = base.enc_off.clone()
        s.cap_off = base.cap_off.clone()
        s.out = torch.empty_like(base.out)
        s.out_len = torch.empty_like(base.out_len)
        s.status = torch.empty_like(base.status)
        slots.append(s)
    for i in range(warmup):
        s = slots[i % R]
        codec.decode_dev(s.enc, s.enc_off, s.out, s.cap_off, s.out_len, s.status)
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for i in range(steps):
        s = slots[i % R]
        codec.decode_dev(s.enc, s.enc_off, s.out, s.cap_off, s.out_len, s.status)
    e1.record()
    torch.cuda.synchronize()
    ms = e0.elapsed_time(e1) / steps
    alg = decode_algorithmic_bytes(b.n, enc_b, b.nbytes)
    return {"workload": b.name, "literals": b.n, "plain_bytes": b.nbytes, "encoded_bytes": enc_b,
            "ms_per_launch": round(ms, 5), "gib_s": round(b.nbytes / (ms / 1e3) / GIB, 3),
            "hbm_frac": round(alg / (ms / 1e3) / 1e9 / HBM_PEAK_GBS, 4), "rotating_copies": R}


class PinnedPool:
    """Output buffers for the host-memory calls: pinned on first use, then
    handed out again in the same order on every later pass (`rewind()`), so
    no timed pass allocates or pins memory."""

    def __init__(self):
        self.bufs, self.i = [], 0

    def rewind(self):
        self.i = 0

    def __call__(self, nbytes):
        import torch

        if self.i == len(self.bufs):
            self.bufs.append(torch.empty(nbytes, dtype=torch.uint8).pin_memory().numpy())
        b = self.bufs[self.i]
        if len(b) < nbytes:
            b = self.bufs[self.i] = torch.empty(nbytes, dtype=torch.uint8).pin_memory().numpy()
        self.i += 1
        return b


def pcie_inclusive(codec, batch):
    """Host-memory entry points, pinned input and output buffers: H2D + kernels + D2H."""
    import torch

    from minhq_amd import hc

    pin = lambda a: torch.from_numpy(a).pin_memory().numpy()  # noqa: E731
    data, off = pin(batch.data), pin(batch.off)
    epool, dpool = PinnedPool(), PinnedPool()
    enc, eoff = codec.encode(data, off, alloc=epool)  # warm: staging buffers and the pinned pool
    cap = pin(hc.capacity_offsets(eoff))
    codec.decode(enc, eoff, cap, alloc=dpool)
    ta = time.perf_counter()
    codec.encode_len(data, off)
    tb = time.perf_counter()
    epool.rewind()
    t0 = time.perf_counter()
    enc, eoff = codec.encode(data, off, alloc=epool)
    t1 = time.perf_counter()
    dpool.rewind()
    t2 = time.perf_counter()
    out, _, out_len, status = codec.decode(enc, eoff, cap, alloc=dpool)
    t3 = time.perf_counter()
    assert not status.any() and np.array_equal(out_len.astype(np.uint64), np.diff(batch.off))
    P = batch.nbytes
    return {"encode_gib_s": round(P / (t1 - t0) / GIB, 3), "decode_gib_s": round(P / (t3 - t2) / GIB, 3),
            "roundtrip_gib_s": round(P / ((t1 - t0) + (t3 - t2)) / GIB, 3),
            "encode_len_only_gib_s": round(P / (tb - ta) / GIB, 3), "literals": batch.n,
            "note": "host-memory ABI (encode = encode_len + host scan + encode), pinned host buffers, "
                    "chunks of ~2 MB pipelined over 4 streams per device, one device"}


def main():
    ap = argparse.ArgumentParser(description=__doc__.split("\n")[0])
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--literals", type=int, default=1 << 20)
    ap.add_argument("--rotate-gib", type=float, default=1.0, help="total bytes of rotating buffer copies")
    ap.add_argument("--cpu-seconds", type=float, default=10.0)
    ap.add_argument("--no-cpu", action="store_true")
    ap.add_argument("--no-extras", action="store_true")
    ap.add_argument("--streams", type=int, default=3, help="streams the batches alternate over")
    ap.add_argument("--traffic", default=os.path.join(REPO, "profiles", "pmc_traffic.json"))
    args = ap.parse_args()

    import torch

    from minhq_amd import build as mbuild
    from minhq_amd import hc, workloads

    if not os.path.exists(mbuild.LIB):
        mbuild.build()
    world, rank, local, pg = dist_setup()
    dev = torch.device("cuda", local)
    codec = hc.Codec(devices=[local])

    batch = workloads.make_batch(args.literals, "uniform", "hdr", workloads.SEED_NORTH_STAR + rank, 8, 64,
                                 f"config2: {args.literals} literals U{{8..64}} hdr")
    enc_b, cap_b = encoded_sizes(codec, batch, dev)
    first = Slot(batch, enc_b, cap_b, dev)
    R = max(2, int(np.ceil(args.rotate_gib * GIB / first.nbytes())))
    slots = [first] + [Slot(batch, enc_b, cap_b, dev) for _ in range(R - 1)]
    for s in slots:  # correctness gate before timing
        round_trip(codec, s)
        verify_slot(s, batch)

    # --streams S: consecutive batches alternate over S streams (batches are
    # independent; a slot always runs on the same stream, so its reuse stays
    # in stream order), letting one batch's first kernels fill the CUs that the
    # previous batch's last kernel leaves idle at its tail
    S = max(1, args.streams)
    streams = [None] if S == 1 else [torch.cuda.Stream(device=dev).cuda_stream for _ in range(S)]
    if R % S:
        slots += [Slot(batch, enc_b, cap_b, dev) for _ in range(S - R % S)]
        R = len(slots)
        for s in slots:
            round_trip(codec, s)
            verify_slot(s, batch)
    for i in range(args.warmup):
        round_trip(codec, slots[i % R], streams[i % S])
    # the timed region: K whole steps, no instrumentation between the kernels
    # (a timing event between two launches costs ~5.7 us of idle GPU)
    barrier(pg)
    t0 = time.perf_counter()
    for i in range(args.steps):
        round_trip(codec, slots[i % R], streams[i % S])
    barrier(pg)
    el = time.perf_counter() - t0
    el_max = max_over_ranks(pg, el)
    for s in slots:  # every slot's last round trip (concurrent streams) is still exact
        verify_slot(s, batch)
    # per-kernel launch durations, live: the same slots, events only around
    # a run of back-to-back launches of one kernel on the launch stream
    enc_ms = kernel_ms(codec, slots, "encode", max(args.steps, 20))
    dec_ms = kernel_ms(codec, slots, "decode", max(args.steps, 20))

    plain_total = batch.nbytes * world * args.steps
    value = plain_total / el_max / GIB
    ms_per_step = el_max / args.steps * 1e3
    alg = decode_algorithmic_bytes(batch.n, enc_b, batch.nbytes)
    achieved = alg / (dec_ms / 1e3) / 1e9
    traffic = load_traffic(args.traffic, "decode_kernel")

    res = {
        "metric": "device-resident Huffman literal GiB/s (encode+decode)",
        "value": round(value, 3),
        "unit": "GiB/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": round(ms_per_step, 4),
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "u8",
        "data": "synthetic",
        "config": {"workload": batch.name, "literals_per_gpu": batch.n, "plain_bytes_per_gpu": batch.nbytes,
                   "encoded_bytes_per_gpu": enc_b, "step": "encode_len+offsets+encode+decode",
                   "rotating_copies": R, "streams": S, "parallelism": f"shard{world} (independent literals, no collective)"},
        "roofline": {"bound": "hbm", "kernel": "decode_kernel", "achieved": round(achieved, 2),
                     "peak": HBM_PEAK_GBS, "unit": "GB/s", "frac": round(achieved / HBM_PEAK_GBS, 4),
                     "traffic": traffic, "alg_bytes_per_launch": alg, "ms_per_launch": round(dec_ms, 5)},
        "encode_ms_per_launch": round(enc_ms, 5),
    }
    if rank == 0 and world == 1 and not args.no_extras:
        res["decode_only_northstar"] = decode_only(codec, dev, max(args.steps, 20), args.warmup,
                                                   args.rotate_gib * GIB)
        res["pcie_inclusive"] = pcie_inclusive(codec, batch)
    if rank == 0 and world == 1 and not args.no_cpu:
        res["cpu_baseline"] = cpu_baseline(batch, args.cpu_seconds)
    if rank == 0:
        print(json.dumps(res), flush=True)
    codec.close()
    if pg is not None:
        pg.destroy_process_group()


if __name__ == "__main__":
    main()
