#!/usr/bin/env python3
"""bench.py -- device-resident Huffman literal GiB/s (encode+decode), 1..8 GPUs.

Metric (BASELINE.json): "device-resident Huffman literal GiB/s (encode+decode)".
Workload (BASELINE.json configs[1]): 2^20 synthetic header-field literals per
GPU, lengths U{8..64}, bytes drawn from the netbsd.qif header-byte histogram
(minhq_amd/workloads.py).  One step = one full round trip of
one batch on the device: the packed encode (sizes, offsets and codes in one
launch, mhq_huff_encode_packed_dev) then the decode (mhq_huff_decode_dev),
both through the C ABI (include/mhq_huff.h), inputs resident in HBM; the two
calls of each slot are bound once (hc.Codec.bound_call), so the host pays per
step about what a cgo caller would, not ctypes' argument conversion.  Rotating
copies of every buffer (>= 1 GiB in all) keep the 256 MB Infinity Cache from
serving a step's inputs from the previous step.

Consecutive batches alternate over 4 HIP streams (--streams; batches are
independent, a slot always runs on the same stream): one batch's first
kernels fill the CUs that the previous batch's decode leaves idle at its tail.

value = plaintext bytes of all ranks x steps / max-over-ranks wall time / 2^30.
Multi-GPU: one process per GPU.  `--gpus N` without a launcher starts N ranks
under torch.distributed.run (a child process, before anything touches a GPU);
under a launcher the ranks come from RANK/LOCAL_RANK/WORLD_SIZE.  Each rank
owns an independent batch (no data-path collective, weak scaling); the
process group carries only the barrier and the max over ranks.

Extra fields (not `value`):
  roofline            the step's dominant (longest) kernel against the HBM
                      roofline; roofline_decode / roofline_encode_packed: both;
  long_run            the same step timed over >= 200 steps;
  decode_only_northstar  2^20 x U{8..56} decode (the north star's shape);
  config4_sharded     one 2^24-literal Zipf batch (BASELINE.json configs[3]),
                      split by encoded bytes over the ranks, each rank decoding
                      its shard device-resident; max over ranks (strong scaling);
  config4 / config5   full-size single-GPU decode, encode and layout times
                      (configs[3] at 2^24, configs[4] at 4 x 2^20 x 128 B), and
                      config 5's PCIe-inclusive decode rate;
  pcie_inclusive      host-memory ABI rates on the headline batch (pinned
                      buffers, read and written in place by the kernels;
                      pageable ones staged), run after configs 4 and 5;
  cpu_baseline        the oracle (minhq's Go algorithm restated in C,
                      oracle/huff_oracle.c; no Go toolchain exists here) on 1
                      thread and on the box's thread share, plus the
                      table-driven CPU decoder beside it.
"""
from __future__ import annotations

import argparse
import json
import os
import socket
import subprocess
import sys
import time

import numpy as np

REPO = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, REPO)

HBM_PEAK_GBS = 8000.0  # MI355X_MICROARCH.md: HBM3E 8.0 TB/s spec
GIB = float(1 << 30)


def log(*a):
    print(*a, file=sys.stderr, flush=True)


def spawn_ranks(n: int) -> int:
    """Runs this script as n ranks under torch.distributed.run (a child
    process: nothing in this process has touched a GPU) and returns its code."""
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={n}",
           "--master-addr", "127.0.0.1", "--master-port", str(port), os.path.abspath(__file__)] + sys.argv[1:]
    env = dict(os.environ, HSA_ENABLE_IPC_MODE_LEGACY=os.environ.get("HSA_ENABLE_IPC_MODE_LEGACY", "0"))
    return subprocess.call(cmd, env=env)


# The process group only carries barriers and one max over ranks (the path has
# no data exchange), so it runs on gloo over the host: an RCCL
# communicator would be initialised on every rank for a handful of scalars.
# MHQ_BENCH_BACKEND=nccl selects RCCL instead; MHQ_BENCH_SHARE_GPU=1 maps rank
# r to GPU r mod (GPUs visible), to rehearse N > 1 on fewer GPUs.
BACKEND = os.environ.get("MHQ_BENCH_BACKEND", "gloo")


def dist_setup():
    import torch

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if os.environ.get("MHQ_BENCH_SHARE_GPU") == "1":
        local %= torch.cuda.device_count()
    torch.cuda.set_device(local)
    pg = None
    if world > 1:
        import torch.distributed as dist

        if BACKEND == "nccl":
            dist.init_process_group("nccl", device_id=torch.device("cuda", local))
        else:
            dist.init_process_group(BACKEND)
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

    return shard.max_over_ranks(pg, x, "cuda" if BACKEND == "nccl" else "cpu")


def sum_over_ranks(pg, x: int) -> int:
    if pg is None:
        return int(x)
    import torch

    t = torch.tensor([int(x)], dtype=torch.int64, device="cuda" if BACKEND == "nccl" else "cpu")
    pg.all_reduce(t, op=pg.ReduceOp.SUM)
    return int(t.item())


class Slot:
    """One rotating copy of every buffer of a round-trip step."""

    def __init__(self, batch, enc_bytes, cap_bytes, dev, packed=False):
        import torch

        n = batch.n
        self.n = n
        self.plain = batch.nbytes
        self.data = torch.from_numpy(batch.data).to(dev)
        self.off = torch.from_numpy(batch.off.view(np.int64)).to(dev)
        self.enc_len = torch.empty(n, dtype=torch.int32, device=dev)
        self.enc_off = torch.empty(n + 1, dtype=torch.int64, device=dev)
        self.cap_off = torch.empty(n + 1, dtype=torch.int64, device=dev)
        # (the packed encode wants room for the most any plaintext encodes to)
        self.enc = torch.empty(max(enc_bytes + 16, 30 * batch.nbytes // 8 + batch.n if packed else 0), dtype=torch.uint8,
                               device=dev)
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


PACKED = True  # --encode packed: the encode side as one call (mhq_huff_encode_packed_dev)


def bind_round_trip(codec, s, stream=None):
    """The step's two calls (packed encode, decode) on slot s, bound once
    (hc.Codec.bound_call): the timed loop then pays a cgo-like host cost per
    call, not ctypes' conversion of a dozen arguments (the
    20-step run lost 14 % to submission)."""
    return (codec.bind_encode_packed_dev(s.data, s.off, s.plain, s.enc_len, s.enc_off, s.cap_off, s.enc,
                                         stream=stream),
            codec.bind_decode_dev(s.enc, s.enc_off, s.out, s.cap_off, s.out_len, s.status, stream=stream))


def round_trip(codec, s, stream=None, bound=None):
    if bound is not None:
        for call in bound:
            call()
        return
    if PACKED:
        # sizes, placement and codes in one launch (enc_packed.hip), decode
        codec.encode_packed_dev(s.data, s.off, s.plain, s.enc_len, s.enc_off, s.cap_off, s.enc, stream=stream)
    else:
        # encode_len + offsets scan (one call, two launches), encode, decode
        codec.encode_layout_dev(s.data, s.off, s.enc_len, s.enc_off, s.cap_off, stream=stream)
        codec.encode_dev(s.data, s.off, s.enc, s.enc_off, stream=stream)
    codec.decode_dev(s.enc, s.enc_off, s.out, s.cap_off, s.out_len, s.status, stream=stream)


def events_ms(fn, launches):
    """Mean duration of fn() over `launches` back-to-back calls on the current
    stream (the one the ABI calls launch on), HIP events at the ends only."""
    import torch

    stream = torch.cuda.current_stream()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record(stream)
    for i in range(launches):
        fn(i)
    e1.record(stream)
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / launches


def kernel_ms(codec, slots, which, launches):
    """Mean duration of one encode or decode launch over back-to-back launches
    rotating through the slots."""
    def run(i):
        s = slots[i % len(slots)]
        if which == "encode":
            codec.encode_dev(s.data, s.off, s.enc, s.enc_off)
        elif which == "packed":
            codec.encode_packed_dev(s.data, s.off, s.plain, s.enc_len, s.enc_off, s.cap_off, s.enc)
        elif which == "layout":
            codec.encode_layout_dev(s.data, s.off, s.enc_len, s.enc_off, s.cap_off)
        else:
            codec.decode_dev(s.enc, s.enc_off, s.out, s.cap_off, s.out_len, s.status)

    for i in range(2):
        run(i)
    return events_ms(run, launches)


def decoded_bytes_match(out, cap_off, data, off):
    """The decoded bytes of every literal (at its capacity offset in `out`)
    equal the plaintext, compared on the device."""
    import torch

    lens = off[1:] - off[:-1]
    total = int(lens.sum().item())
    if total == 0:
        return True
    rep = torch.repeat_interleave(cap_off[:-1] - cap_off[0], lens)
    within = torch.arange(total, device=lens.device) - torch.repeat_interleave(torch.cumsum(lens, 0) - lens, lens)
    p0 = int(off[0].item())
    return torch.equal(out[rep + within], data[p0:p0 + total])


def verify_slot(s):
    """The headline's correctness gate: status, lengths and the decoded bytes
    of the slot's last round trip."""
    import torch

    torch.cuda.synchronize()
    assert int(s.status.sum().item()) == 0, "decode reported INVALID on encoder output"
    assert torch.equal(s.out_len.long(), s.off[1:] - s.off[:-1]), "round trip length mismatch"
    assert decoded_bytes_match(s.out, s.cap_off, s.data, s.off), "round trip byte mismatch"


def decode_algorithmic_bytes(n, enc_bytes, plain_bytes):
    # sum C + sum out_len + 8(n+1) in_off + 8(n+1) out_off + 4n out_len + 1n status
    return enc_bytes + plain_bytes + 16 * (n + 1) + 5 * n


def encode_algorithmic_bytes(n, enc_bytes, plain_bytes):
    # SURVEY.md §8d / BASELINE.md: sum L + sum C + 8(n+1) in_off + 8(n+1) out_off + 4n enc_len
    return plain_bytes + enc_bytes + 16 * (n + 1) + 4 * n


def packed_algorithmic_bytes(n, enc_bytes, plain_bytes):
    # the one-launch encode side: sum L + sum C + 8(n+1) in_off + 4n enc_len + 8(n+1) out_off + 8(n+1) cap_off
    return plain_bytes + enc_bytes + 24 * (n + 1) + 4 * n


def layout_algorithmic_bytes(n, plain_bytes):
    # encode_len reads the plaintext and in_off, writes enc_len; the scan writes out_off and cap_off
    return plain_bytes + 8 * (n + 1) + 4 * n + 16 * (n + 1)


def load_traffic(path, kernel):
    try:
        with open(path) as f:
            d = json.load(f)
        return d.get(kernel, {}).get("hbm_bytes_per_launch")
    except Exception:
        return None


def _affinity():
    try:
        return len(os.sched_getaffinity(0))
    except Exception:
        return os.cpu_count() or 1


def _cpu_quota():
    """CPUs' worth of time the cgroup grants this process (cpu.max, cgroup
    v2; cfs quota, v1), or None when unlimited / unknown: the GPU box's
    affinity mask spans every core of the host, its quota does not."""
    try:
        q, p = open("/sys/fs/cgroup/cpu.max").read().split()[:2]
        return None if q == "max" else max(1, round(int(q) / int(p)))
    except Exception:
        pass
    try:
        q = int(open("/sys/fs/cgroup/cpu/cpu.cfs_quota_us").read())
        p = int(open("/sys/fs/cgroup/cpu/cpu.cfs_period_us").read())
        return None if q <= 0 else max(1, round(q / p))
    except Exception:
        return None


def _threads():
    """(threads, where the count comes from): OMP_NUM_THREADS when set -- the
    GPU box sets it to 16, this process's share of a host whose affinity mask
    spans every core -- else the CPU affinity of this process."""
    env = os.environ.get("OMP_NUM_THREADS")
    if env and env.isdigit() and int(env) > 0:
        return int(env), "OMP_NUM_THREADS"
    return _affinity(), "sched_getaffinity"


def _cpu_sample(batch, m):
    """The first m literals of a batch, encoded by the oracle: (plain bytes,
    data, off, enc, enc_off, cap_off)."""
    from minhq_amd import hc
    from oracle import oracle

    m = min(batch.n, m)
    off = batch.off[: m + 1].copy()
    data = batch.data[int(off[0]): int(off[-1])].copy()
    off -= off[0]
    enc_len = oracle.encode_len_batch(data, off, _affinity())
    eoff = np.zeros(m + 1, dtype=np.uint64)
    eoff[1:] = np.cumsum(enc_len, dtype=np.uint64)
    enc = oracle.encode_batch(data, off, eoff, _affinity())
    return int(off[-1]), data, off, enc, eoff, hc.capacity_offsets(eoff)


def _rate(fn, plain, budget):
    """GiB/s of plaintext of fn() repeated for about `budget` seconds."""
    done, t0 = 0, time.perf_counter()
    while True:
        fn()
        done += 1
        el = time.perf_counter() - t0
        if el >= budget:
            return round(plain * done / el / GIB, 4), done, round(el, 2)


def cpu_baseline(batch, seconds: float):
    """The oracle (minhq's Go algorithm restated in C) on the host cores, as
    BASELINE.md asks: config 2 encode+decode on every CPU of this process's
    affinity (std::thread-style pthreads, one contiguous range of literals
    each), on the box's OMP_NUM_THREADS share and on one thread; decode legs
    for the north star and configs 3, 4 and 5 on one thread and on every
    affinity CPU; the table-driven C decoder beside each.  Bounded samples
    (first 2^17 literals; config 5 2^15 x 128 B), about `seconds` in all."""
    from minhq_amd import workloads
    from oracle import oracle

    oracle.build()
    allc = _affinity()
    share, share_src = _threads()
    leg = max(seconds / 20.0, 0.3)
    plain, data, off, enc, eoff, cap = _cpu_sample(batch, 1 << 17)
    m = len(off) - 1

    def roundtrip(th):
        def f():
            el = oracle.encode_len_batch(data, off, th)
            eo = np.zeros(m + 1, dtype=np.uint64)
            eo[1:] = np.cumsum(el, dtype=np.uint64)
            e = oracle.encode_batch(data, off, eo, th)
            oracle.decode_batch(e, eo, cap, th)
        return f

    v_all, n_all, t_all = _rate(roundtrip(allc), plain, 2 * leg)
    v_share, n_share, t_share = _rate(roundtrip(share), plain, leg)
    v_one, n_one, t_one = _rate(roundtrip(1), plain, leg)
    legs = {}
    for name, b, mm in (("northstar", workloads.north_star(1 << 17), 1 << 17),
                        ("config2", batch, 1 << 17),
                        ("config3", workloads.config3(1 << 17), 1 << 17),
                        ("config4", workloads.make_batch(1 << 17, "zipf", "hdr", workloads.SEED_ZIPF), 1 << 17),
                        ("config5", workloads.make_batch(1 << 15, "fixed", "adv", workloads.SEED_ADV, 128, 128),
                         1 << 15)):
        pl, _, _, e, eo, co = _cpu_sample(b, mm)
        legs[name] = {
            "sample": f"first {min(b.n, mm)} literals ({pl} plaintext bytes)",
            "restated_go_1_thread": _rate(lambda: oracle.decode_batch(e, eo, co, 1), pl, leg / 2)[0],
            f"restated_go_{share}_threads": _rate(lambda: oracle.decode_batch(e, eo, co, share), pl, leg / 2)[0],
            f"restated_go_{allc}_threads": _rate(lambda: oracle.decode_batch(e, eo, co, allc), pl, leg / 2)[0],
            f"table_driven_{share}_threads": _rate(lambda: oracle.decode_batch(e, eo, co, share, fast=True), pl,
                                                   leg / 2)[0],
            "unit": "GiB/s of plaintext (decode)"}
    # the reported value: the better of the affinity-wide and the share legs
    # (on the GPU box the affinity mask spans the host's 256 CPUs but the
    # cgroup grants ~16 CPUs of time, so 256 threads thrash: both are shown)
    best_all = v_all >= v_share or share == allc
    quota = _cpu_quota()
    return {"value": v_all if best_all else v_share, "unit": "GiB/s", "cores": allc if best_all else share,
            "kind": "port",
            "cores_source": ("sched_getaffinity (every CPU this process may run on, BASELINE.md: all nproc cores)"
                             if best_all else f"{share_src}: the affinity-wide leg (all {allc} CPUs) ran slower, "
                             f"the cgroup granting {quota} CPUs of time"),
            "affinity_cpus": allc, "cgroup_quota_cpus": quota, "os_cpu_count": os.cpu_count(),
            "sample": f"config 2, first {m} literals of the workload, encode+decode (minhq hc/huffman.go + "
                      f"io/bitio.go bit-serial algorithm restated in C, oracle/huff_oracle.c), pthreads over "
                      f"contiguous literal ranges",
            "affinity": {"value": v_all, "threads": allc, "passes": n_all, "seconds": round(t_all, 2)},
            "share": {"value": v_share, "threads": share, "threads_source": share_src, "passes": n_share,
                      "seconds": round(t_share, 2), "note": "the GPU box's per-GPU CPU share"},
            "single_thread": {"value": v_one, "unit": "GiB/s", "passes": n_one, "seconds": t_one},
            "decode_legs": legs,
            "note": "table-driven: a 12-bit LUT per code, tree walk for longer codes and the literal end "
                    "(orc_huff_decode_fast); same results as the restated loop (tests/test_oracle.py)"}


class Dev:
    """Device-resident copies of one batch and its encoded form."""

    def __init__(self, codec, data, off, dev, encode=True):
        import torch

        self.codec, self.data, self.off = codec, data, off
        n = off.numel() - 1
        self.n = n
        self.plain = int((off[-1] - off[0]).item())
        self.enc_len = torch.empty(max(n, 1), dtype=torch.int32, device=dev)
        self.enc_off = torch.empty(n + 1, dtype=torch.int64, device=dev)
        self.cap_off = torch.empty(n + 1, dtype=torch.int64, device=dev)
        codec.encode_layout_dev(data, off, self.enc_len, self.enc_off, self.cap_off)
        torch.cuda.synchronize()
        self.enc_bytes = int(self.enc_off[-1].item())
        self.cap_bytes = int(self.cap_off[-1].item())
        self.enc = torch.empty(self.enc_bytes + 16, dtype=torch.uint8, device=dev)
        if encode:
            self.encode_range(0, n)

    def encode_range(self, lo, hi):
        """Encodes literals [lo, hi) into their place in self.enc (a rank
        encodes only the shard it decodes)."""
        import torch

        if hi > lo:
            self.codec.encode_dev(self.data, self.off[lo:hi + 1], self.enc, self.enc_off[lo:hi + 1])
        torch.cuda.synchronize()


def decode_slots(dv, lo, hi, rotate_bytes, dev):
    """Rotating decode buffers for literals [lo, hi) of a Dev batch: the
    encoded bytes and rebased offsets copied R times (R copies >= rotate_bytes)."""
    import torch

    a, b = int(dv.enc_off[lo].item()), int(dv.enc_off[hi].item())
    ca, cb = int(dv.cap_off[lo].item()), int(dv.cap_off[hi].item())
    per = (b - a) + (cb - ca) + 16 * (hi - lo + 1) + 5 * (hi - lo)
    R = max(1, int(np.ceil(rotate_bytes / max(per, 1))))
    slots = []
    for _ in range(R):
        s = type("S", (), {})()
        s.enc = dv.enc[a:b + 16].clone()
        s.enc_off = dv.enc_off[lo:hi + 1] - a
        s.cap_off = dv.cap_off[lo:hi + 1] - ca
        s.out = torch.empty(cb - ca + 16, dtype=torch.uint8, device=dev)
        s.out_len = torch.empty(max(hi - lo, 1), dtype=torch.int32, device=dev)
        s.status = torch.empty(max(hi - lo, 1), dtype=torch.uint8, device=dev)
        slots.append(s)
    return slots


def check_decode(dv, lo, hi, s):
    """The decode of literals [lo, hi) reproduces the plaintext (on the device)."""
    import torch

    torch.cuda.synchronize()
    n = hi - lo
    if n == 0:
        return
    assert int(s.status[:n].sum().item()) == 0, "INVALID on encoder output"
    lens = (dv.off[lo + 1:hi + 1] - dv.off[lo:hi])
    assert torch.equal(s.out_len[:n].long(), lens), "length mismatch"
    assert decoded_bytes_match(s.out, s.cap_off, dv.data, dv.off[lo:hi + 1]), "byte mismatch"


def config4_sharded(codec, dev, world, rank, pg, launches, rotate_bytes):
    """BASELINE.json configs[3]: one 2^24-literal Zipf batch split over the
    ranks by encoded bytes; each rank decodes its shard device-resident."""
    import torch

    from minhq_amd import shard, workloads

    n = 1 << 24
    # every rank generates the batch (on its device, seconds) and cuts it by
    # plaintext bytes; only its own shard goes through encode_len, the scan
    # and encode (hdr bytes code at a near-constant ~5.8 bits, so the cut
    # balances the encoded bytes the decode reads as well)
    data, off = workloads.make_batch_device(n, "zipf", "hdr", workloads.SEED_ZIPF, device=dev)
    parts = shard.plan_shards_device(off, world)
    lo, hi = parts[rank]
    s_off = off[lo:hi + 1] - off[lo]
    s_data = data[int(off[lo].item()):int(off[hi].item())]
    dv = Dev(codec, s_data, s_off, dev)
    slots = decode_slots(dv, 0, hi - lo, rotate_bytes, dev)

    def run(i):
        s = slots[i % len(slots)]
        codec.decode_dev(s.enc, s.enc_off, s.out, s.cap_off, s.out_len, s.status)

    run(0)
    check_decode(dv, 0, hi - lo, slots[0])
    barrier(pg)
    ms = events_ms(run, launches)
    barrier(pg)
    ms_max = max_over_ranks(pg, ms)
    plain_all = int((off[-1] - off[0]).item())
    enc_total = sum_over_ranks(pg, dv.enc_bytes)
    alg = decode_algorithmic_bytes(n, enc_total, plain_all)
    res = {"workload": f"config4: {n} literals Zipf{{4..256}} hdr, one batch split by plaintext bytes",
           "literals": n, "plain_bytes": plain_all, "encoded_bytes": enc_total, "ranks": world,
           "shard_literals_rank0": parts[0][1] - parts[0][0],
           "ms_per_launch_max_over_ranks": round(ms_max, 5),
           "shard_encoded_bytes_rank0": dv.enc_bytes,
           "gib_s": round(plain_all / (ms_max / 1e3) / GIB, 2),
           "hbm_frac_aggregate": round(alg / (ms_max / 1e3) / 1e9 / (HBM_PEAK_GBS * world), 4),
           "scaling": "strong", "rotating_copies": len(slots)}
    if world == 1:  # full-size single-GPU times of the other kernels (the shard is the whole batch)
        plain_alg = layout_algorithmic_bytes(n, dv.plain)
        enc_ms = events_ms(lambda i: codec.encode_dev(s_data, s_off, dv.enc, dv.enc_off), max(4, launches // 2))
        lay_ms = events_ms(lambda i: codec.encode_layout_dev(s_data, s_off, dv.enc_len, dv.enc_off, dv.cap_off),
                           max(4, launches // 2))
        res["decode_hbm_frac"] = round(alg / (ms / 1e3) / 1e9 / HBM_PEAK_GBS, 4)
        res["encode_ms"] = round(enc_ms, 5)
        res["encode_hbm_frac"] = round(encode_algorithmic_bytes(n, dv.enc_bytes, dv.plain) / (enc_ms / 1e3) / 1e9
                                       / HBM_PEAK_GBS, 4)
        res["layout_ms"] = round(lay_ms, 5)
        res["layout_hbm_frac"] = round(plain_alg / (lay_ms / 1e3) / 1e9 / HBM_PEAK_GBS, 4)
    del slots, dv, data, off, s_data, s_off
    torch.cuda.empty_cache()
    return res


def config5(codec, dev, launches, rotate_bytes):
    """BASELINE.json configs[4]: 4 x 2^20 literals of 128 bytes whose codes are
    >= 26 bits; 1-GPU decode roofline and the PCIe-inclusive decode rate."""
    import torch

    from minhq_amd import hc, workloads

    n = 4 << 20
    data, off = workloads.make_batch_device(n, "fixed", "adv", workloads.SEED_ADV, 128, 128, device=dev)
    dv = Dev(codec, data, off, dev)
    slots = decode_slots(dv, 0, n, rotate_bytes, dev)

    def run(i):  # (the batch's encoded size given: mhq_huff_decode_sized_dev picks the long-literal form)
        s = slots[i % len(slots)]
        codec.decode_dev(s.enc, s.enc_off, s.out, s.cap_off, s.out_len, s.status, in_bytes=dv.enc_bytes)

    run(0)
    check_decode(dv, 0, n, slots[0])
    ms = events_ms(run, launches)
    alg = decode_algorithmic_bytes(n, dv.enc_bytes, dv.plain)
    enc_ms = events_ms(lambda i: codec.encode_dev(data, off, dv.enc, dv.enc_off), max(4, launches // 2))
    lay_ms = events_ms(lambda i: codec.encode_layout_dev(data, off, dv.enc_len, dv.enc_off, dv.cap_off),
                       max(4, launches // 2))
    res = {"workload": f"config5: {n} literals x 128 B, bytes with >= 26-bit codes", "literals": n,
           "plain_bytes": dv.plain, "encoded_bytes": dv.enc_bytes,
           "decode_ms": round(ms, 5), "decode_gib_s": round(dv.plain / (ms / 1e3) / GIB, 2),
           "decode_hbm_frac": round(alg / (ms / 1e3) / 1e9 / HBM_PEAK_GBS, 4),
           "encode_ms": round(enc_ms, 5),
           "encode_hbm_frac": round(encode_algorithmic_bytes(n, dv.enc_bytes, dv.plain) / (enc_ms / 1e3) / 1e9
                                    / HBM_PEAK_GBS, 4),
           "layout_ms": round(lay_ms, 5), "rotating_copies": len(slots)}
    # PCIe-inclusive decode: pinned host input (encoded bytes, offsets), pinned host outputs
    enc_h = torch.empty(dv.enc_bytes, dtype=torch.uint8).pin_memory()
    enc_h.copy_(dv.enc[:dv.enc_bytes])
    eoff_h = torch.empty(n + 1, dtype=torch.int64).pin_memory()
    eoff_h.copy_(dv.enc_off)
    cap_h = torch.empty(n + 1, dtype=torch.int64).pin_memory()
    cap_h.copy_(dv.cap_off)
    out_h = torch.empty(dv.cap_bytes + 16, dtype=torch.uint8).pin_memory()
    len_h = torch.empty(n, dtype=torch.int32).pin_memory()
    st_h = torch.empty(n, dtype=torch.uint8).pin_memory()
    del slots
    torch.cuda.empty_cache()
    pool = iter([out_h.numpy(), len_h.numpy().view(np.uint8), st_h.numpy()] * 2)
    alloc = lambda nb: next(pool)  # noqa: E731  (the pinned outputs, in the order decode asks for them)
    e, eo, co = enc_h.numpy(), eoff_h.numpy().view(np.uint64), cap_h.numpy().view(np.uint64)
    codec.decode(e, eo, co, alloc=alloc)  # warm: staging buffers
    t0 = time.perf_counter()
    _, _, out_len, status = codec.decode(e, eo, co, alloc=alloc)
    t1 = time.perf_counter()
    assert not status.any() and np.array_equal(out_len.astype(np.int64), np.full(n, 128))
    res["pcie_inclusive_decode_gib_s"] = round(dv.plain / (t1 - t0) / GIB, 3)
    res["pcie_note"] = "host-memory mhq_huff_decode, pinned input and outputs read and written in place over PCIe"
    del dv, data, off
    torch.cuda.empty_cache()
    return res


def decode_only(codec, dev, steps, warmup, rotate_bytes, b=None):
    """Decode-only rate of one 2^20-literal batch: by default the north star's
    2^20 x U{8..56} hdr literals."""
    import torch

    from minhq_amd import workloads

    b = b if b is not None else workloads.north_star()
    data = torch.from_numpy(b.data).to(dev)
    off = torch.from_numpy(b.off.view(np.int64)).to(dev)
    dv = Dev(codec, data, off, dev)
    slots = decode_slots(dv, 0, b.n, rotate_bytes, dev)

    def run(i):
        s = slots[i % len(slots)]
        codec.decode_dev(s.enc, s.enc_off, s.out, s.cap_off, s.out_len, s.status)

    run(0)
    check_decode(dv, 0, b.n, slots[0])
    for i in range(warmup):
        run(i)
    ms = events_ms(run, steps)
    alg = decode_algorithmic_bytes(b.n, dv.enc_bytes, b.nbytes)
    return {"workload": b.name, "literals": b.n, "plain_bytes": b.nbytes, "encoded_bytes": dv.enc_bytes,
            "ms_per_launch": round(ms, 5), "gib_s": round(b.nbytes / (ms / 1e3) / GIB, 3),
            "hbm_frac": round(alg / (ms / 1e3) / 1e9 / HBM_PEAK_GBS, 4), "alg_bytes_per_launch": alg,
            "rotating_copies": len(slots)}


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
    """Host-memory entry points, pinned input and output buffers (read and
    written in place by the kernels): two warm calls of each (the pinned pool
    allocated, then the GPU's first touches of its pages), then three timed
    calls each; the rates are the medians, every call listed."""
    import torch

    from minhq_amd import hc

    pin = lambda a: torch.from_numpy(a).pin_memory().numpy()  # noqa: E731
    data, off = pin(batch.data), pin(batch.off)
    epool, dpool, lpool = PinnedPool(), PinnedPool(), PinnedPool()
    P = batch.nbytes

    def timed(fn, pool, reps=3, warm=2):
        ts = []
        for r in range(warm + reps):
            pool.rewind()
            t0 = time.perf_counter()
            res = fn()
            if r >= warm:
                ts.append(time.perf_counter() - t0)
        return res, ts

    rate = lambda ts: round(P / float(np.median(ts)) / GIB, 3)  # noqa: E731
    each = lambda ts: [round(P / t / GIB, 3) for t in ts]  # noqa: E731
    (enc, eoff), te = timed(lambda: codec.encode(data, off, alloc=epool), epool)
    enc, eoff = pin(np.array(enc)), pin(np.array(eoff))
    cap = pin(hc.capacity_offsets(eoff))
    _, tl = timed(lambda: codec.encode_len(data, off, alloc=lpool), lpool)
    (out, _, out_len, status), td = timed(lambda: codec.decode(enc, eoff, cap, alloc=dpool), dpool)
    assert not status.any() and np.array_equal(out_len.astype(np.uint64), np.diff(batch.off))
    # the staged fallback: pageable buffers (copied through pinned staging)
    e_pg, o_pg, c_pg = np.array(enc), np.array(eoff), np.array(cap)
    tp0 = time.perf_counter()
    _, _, pl, ps = codec.decode(e_pg, o_pg, c_pg)
    tp1 = time.perf_counter()
    assert not ps.any() and np.array_equal(pl.astype(np.uint64), np.diff(batch.off))
    return {"encode_gib_s": rate(te), "decode_gib_s": rate(td),
            "roundtrip_gib_s": round(P / (float(np.median(te)) + float(np.median(td))) / GIB, 3),
            "encode_len_only_gib_s": rate(tl),
            "encode_calls_gib_s": each(te), "decode_calls_gib_s": each(td), "encode_len_calls_gib_s": each(tl),
            "pageable_decode_gib_s": round(P / (tp1 - tp0) / GIB, 3), "literals": batch.n,
            "note": "host-memory ABI (encode = encode_len + host scan + encode), pinned host buffers: the kernels "
                    "read and write them in place over PCIe (one launch per device); medians of 3 calls after 2 "
                    "warm ones; pageable buffers go through 2 MB chunks staged over 4 streams (one call); run "
                    "after configs 4 and 5"}


def main():
    ap = argparse.ArgumentParser(description=__doc__.split("\n")[0])
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=200)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--literals", type=int, default=1 << 20)
    ap.add_argument("--rotate-gib", type=float, default=1.0, help="total bytes of rotating buffer copies")
    ap.add_argument("--cpu-seconds", type=float, default=16.0)
    ap.add_argument("--long-steps", type=int, default=2000, help="steps of the extra long_run timing (0: skip)")
    ap.add_argument("--no-cpu", action="store_true")
    ap.add_argument("--no-extras", action="store_true")
    ap.add_argument("--no-configs", action="store_true", help="skip the full-size configs 4 and 5")
    ap.add_argument("--encode", choices=["packed", "split"], default="packed",
                    help="the step's encode side: one call (packed) or the layout call + encode (split)")
    ap.add_argument("--streams", type=int, default=4, help="streams the batches alternate over (4: the hardware queues a process gets)")
    ap.add_argument("--traffic", default=os.path.join(REPO, "profiles", "pmc_traffic.json"))
    args = ap.parse_args()

    if args.gpus > 1 and "WORLD_SIZE" not in os.environ:
        raise SystemExit(spawn_ranks(args.gpus))

    import torch

    from minhq_amd import build as mbuild
    from minhq_amd import hc, workloads

    if not os.path.exists(mbuild.LIB):
        mbuild.build()
    world, rank, local, pg = dist_setup()
    if world != args.gpus and rank == 0:
        log(f"bench.py: --gpus {args.gpus} but WORLD_SIZE={world}; measuring {world} rank(s)")
    dev = torch.device("cuda", local)
    codec = hc.Codec(devices=[local])

    batch = workloads.make_batch(args.literals, "uniform", "hdr", workloads.SEED_NORTH_STAR + rank, 8, 64,
                                 f"config2: {args.literals} literals U{{8..64}} hdr")
    global PACKED
    PACKED = args.encode == "packed"
    enc_b, cap_b = encoded_sizes(codec, batch, dev)
    first = Slot(batch, enc_b, cap_b, dev, PACKED)
    R = max(2, int(np.ceil(args.rotate_gib * GIB / first.nbytes())))
    slots = [first] + [Slot(batch, enc_b, cap_b, dev, PACKED) for _ in range(R - 1)]
    for s in slots:  # correctness gate before timing
        round_trip(codec, s)
        verify_slot(s)

    # --streams S: consecutive batches alternate over S streams (batches are
    # independent; a slot always runs on the same stream, so its reuse stays
    # in stream order), letting one batch's first kernels fill the CUs that the
    # previous batch's last kernel leaves idle at its tail
    S = max(1, args.streams)
    streams = [None] if S == 1 else [torch.cuda.Stream(device=dev).cuda_stream for _ in range(S)]
    if R % S:
        slots += [Slot(batch, enc_b, cap_b, dev, PACKED) for _ in range(S - R % S)]
        R = len(slots)
        for s in slots:
            round_trip(codec, s)
            verify_slot(s)
    # slot i % R always runs on stream i % S (R is a multiple of S): its calls bound once
    bound = [bind_round_trip(codec, slots[i], streams[i % S]) if PACKED else None for i in range(R)]
    for i in range(args.warmup):
        round_trip(codec, slots[i % R], streams[i % S], bound[i % R])
    # the timed region: K whole steps, no instrumentation between the kernels
    # (a timing event between two launches costs ~5.7 us of idle GPU)
    barrier(pg)
    t0 = time.perf_counter()
    for i in range(args.steps):
        round_trip(codec, slots[i % R], streams[i % S], bound[i % R])
    barrier(pg)
    el = time.perf_counter() - t0
    el_max = max_over_ranks(pg, el)
    for s in slots:  # every slot's last round trip (concurrent streams) is still exact
        verify_slot(s)
    long_run = None
    if args.long_steps > 0 and not args.no_extras:
        barrier(pg)
        t0 = time.perf_counter()
        for i in range(args.long_steps):
            round_trip(codec, slots[i % R], streams[i % S], bound[i % R])
        barrier(pg)
        el_long = max_over_ranks(pg, time.perf_counter() - t0)
        for s in slots:
            verify_slot(s)
        long_run = {"steps": args.long_steps, "seconds": round(el_long, 5),
                    "value": round(batch.nbytes * world * args.long_steps / el_long / GIB, 3),
                    "ms_per_step": round(el_long / args.long_steps * 1e3, 5)}
    # per-kernel launch durations, live: the same slots, events only around
    # a run of back-to-back launches of one kernel on the launch stream
    enc_ms = kernel_ms(codec, slots, "encode", max(args.steps, 50))
    lay_ms = kernel_ms(codec, slots, "layout", max(args.steps, 50))
    pk_ms = kernel_ms(codec, slots, "packed", max(args.steps, 50)) if PACKED else None
    dec_ms = kernel_ms(codec, slots, "decode", max(args.steps, 50))

    plain_total = batch.nbytes * world * args.steps
    value = plain_total / el_max / GIB
    ms_per_step = el_max / args.steps * 1e3
    alg = decode_algorithmic_bytes(batch.n, enc_b, batch.nbytes)
    achieved = alg / (dec_ms / 1e3) / 1e9
    traffic = load_traffic(args.traffic, "decode_kernel")
    roof_dec = {"bound": "hbm", "kernel": "decode", "achieved": round(achieved, 2),
                "peak": HBM_PEAK_GBS, "unit": "GB/s", "frac": round(achieved / HBM_PEAK_GBS, 4),
                "traffic": traffic, "traffic_source": os.path.relpath(args.traffic, REPO),
                "alg_bytes_per_launch": alg, "ms_per_launch": round(dec_ms, 5)}
    roof_pk = None
    if pk_ms is not None:
        pk_alg = packed_algorithmic_bytes(batch.n, enc_b, batch.nbytes)
        pk_ach = pk_alg / (pk_ms / 1e3) / 1e9
        roof_pk = {"bound": "hbm", "kernel": "encode_packed", "achieved": round(pk_ach, 2),
                   "peak": HBM_PEAK_GBS, "unit": "GB/s", "frac": round(pk_ach / HBM_PEAK_GBS, 4),
                   "traffic": load_traffic(args.traffic, "encode_packed_kernel"),
                   "traffic_source": os.path.relpath(args.traffic, REPO),
                   "alg_bytes_per_launch": pk_alg, "ms_per_launch": round(pk_ms, 5)}
    # `roofline`: the step's dominant (longest) kernel; both are reported
    dominant = roof_pk if roof_pk is not None and pk_ms > dec_ms else roof_dec

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
                   "encoded_bytes_per_gpu": enc_b,
                   "step": "encode_packed+decode" if PACKED else "encode_len+offsets+encode+decode",
                   "rotating_copies": R, "streams": S, "parallelism": f"shard{world} (independent literals, no collective)"},
        "roofline": dominant,
        "roofline_decode": roof_dec,
        "roofline_encode_packed": roof_pk,
        "encode_ms_per_launch": round(enc_ms, 5),
        "layout_ms_per_call": round(lay_ms, 5),
        "packed_encode_ms_per_call": round(pk_ms, 5) if pk_ms is not None else None,
        "encode_hbm_frac": round(encode_algorithmic_bytes(batch.n, enc_b, batch.nbytes) / (enc_ms / 1e3) / 1e9
                                 / HBM_PEAK_GBS, 4),
    }
    if long_run:
        res["long_run"] = long_run
    del slots
    torch.cuda.empty_cache()
    if not args.no_extras and not args.no_configs:
        res["config4_sharded"] = config4_sharded(codec, dev, world, rank, pg, max(args.steps, 20),
                                                 args.rotate_gib * GIB)
    if rank == 0 and world == 1 and not args.no_extras:
        res["decode_only_northstar"] = decode_only(codec, dev, max(args.steps, 50), args.warmup,
                                                   args.rotate_gib * GIB)
        # the other 2^20 shapes SURVEY.md §8(d) names: config 2 with printable
        # bytes (codes up to 15 bits) and config 3 (the QIF corpus literals)
        res["decode_only_shapes"] = {
            "config2_print": decode_only(codec, dev, max(args.steps, 50), args.warmup, args.rotate_gib * GIB,
                                         workloads.config2(1 << 20, "print")),
            "config3_qif": decode_only(codec, dev, max(args.steps, 50), args.warmup, args.rotate_gib * GIB,
                                       workloads.config3(1 << 20))}
        if not args.no_configs:
            res["config5"] = config5(codec, dev, max(args.steps, 10), args.rotate_gib * GIB)
        # the host-memory (PCIe-inclusive) rates last: after configs 4 and 5
        # have allocated and freed gigabytes (host path)
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
