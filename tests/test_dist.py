"""Multi-rank path on CPU: gloo, world_size 2.

The GPU path shards literals across ranks with no data-path collective; the
process group carries only the barrier and the max-over-ranks timing.  These
tests run that control flow with gloo: each rank takes its byte-balanced
shard, decodes it (the CPU oracle stands in for the device here -- test
infrastructure only), and the gathered shards must equal the whole batch.
"""
import os
import socket

import numpy as np
import pytest

from minhq_amd import shard, workloads

torch = pytest.importorskip("torch")
import torch.distributed as dist  # noqa: E402
import torch.multiprocessing as mp  # noqa: E402


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def test_plan_shards_balanced_and_contiguous():
    b = workloads.make_batch(5000, "zipf", "hdr", 7, 4, 256, "zipf")
    for parts in (1, 2, 3, 8):
        r = shard.plan_shards(b.off, parts)
        assert r[0][0] == 0 and r[-1][1] == b.n
        assert all(r[k][1] == r[k + 1][0] for k in range(parts - 1))
        sizes = [int(b.off[hi] - b.off[lo]) for lo, hi in r]
        assert sum(sizes) == b.nbytes
        assert max(sizes) - min(sizes) <= 2 * 256  # each cut is within one literal of its target


def test_plan_shards_edge_cases():
    assert shard.plan_shards(np.zeros(1, np.uint64), 4) == [(0, 0)] * 4
    off = np.array([0, 10], dtype=np.uint64)
    r = shard.plan_shards(off, 3)
    assert sum(hi - lo for lo, hi in r) == 1
    with pytest.raises(ValueError):
        shard.plan_shards(off, 0)


def test_shard_view_and_gather_round_trip():
    b = workloads.make_batch(1000, "uniform", "print", 3, 0, 40, "u")
    parts = shard.plan_shards(b.off, 4)
    offs, datas = [], []
    for lo, hi in parts:
        d, o = shard.shard_view(b.data, b.off, lo, hi)
        assert int(o[0]) == 0 and len(d) == int(o[-1])
        offs.append(o)
        datas.append(d)
    assert np.array_equal(shard.gather_offsets(offs), b.off - b.off[0])
    assert np.array_equal(np.concatenate(datas), b.data)


def _worker(rank, world, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from oracle import oracle

        b = workloads.make_batch(3000, "uniform", "hdr", workloads.SEED_NORTH_STAR, 8, 56, "ns")
        # the batch is encoded once (identically on every rank), then sharded by encoded bytes
        enc_len = oracle.encode_len_batch(b.data, b.off, 1)
        eoff = np.zeros(b.n + 1, dtype=np.uint64)
        eoff[1:] = np.cumsum(enc_len, dtype=np.uint64)
        enc = oracle.encode_batch(b.data, b.off, eoff, 1)
        lo, hi = shard.plan_shards(eoff, world)[rank]
        d, o = shard.shard_view(enc, eoff, lo, hi)
        from minhq_amd import hc

        cap = hc.capacity_offsets(o)
        out, out_len, status = oracle.decode_batch(d, o, cap, 1)
        lits = [bytes(out[int(cap[i]):int(cap[i]) + int(out_len[i])]) for i in range(hi - lo)]
        gathered = [None] * world
        dist.all_gather_object(gathered, (lo, hi, lits, int(status.sum())))
        t = shard.max_over_ranks(dist, float(rank + 1))
        dist.barrier()
        if rank == 0:
            whole = [x for part in sorted(gathered) for x in part[2]]
            want = [bytes(b.data[int(b.off[i]):int(b.off[i + 1])]) for i in range(b.n)]
            q.put((whole == want, sum(p[3] for p in gathered), t, [p[:2] for p in sorted(gathered)]))
    finally:
        dist.destroy_process_group()


def test_two_rank_gloo_shard_decode_gather():
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    ok, bad, tmax, ranges = q.get(timeout=180)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    assert ok and bad == 0
    assert tmax == 2.0  # max over ranks
    assert ranges[0][0] == 0 and ranges[0][1] == ranges[1][0] and ranges[1][1] == 3000


def test_plan_shards_device_matches_host():
    """bench.py's config-4 split (shard.plan_shards_device, on the device's
    offsets) equals the host planner."""
    b = workloads.make_batch(20000, "zipf", "hdr", workloads.SEED_ZIPF)
    off_t = torch.from_numpy(b.off.view(np.int64).copy())
    for parts in (1, 2, 3, 8):
        assert shard.plan_shards_device(off_t, parts) == shard.plan_shards(b.off, parts)
    assert shard.plan_shards_device(torch.zeros(1, dtype=torch.int64), 4) == [(0, 0)] * 4
