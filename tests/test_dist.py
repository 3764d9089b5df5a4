"""Multi-rank path: gloo, world_size 2.

The GPU path shards literals across ranks with no data-path collective; the
process group carries only the barrier and the max-over-ranks timing.  These
tests run that control flow with gloo: each rank takes its byte-balanced
shard, decodes it, and the gathered shards must equal the whole batch.  On
CPU the oracle stands in for the device (test infrastructure only);
`test_two_rank_gloo_hip_decode` (-m gpu) runs the same with both ranks
decoding through libmhq_huff.so on device 0.
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


def _hip_worker(rank, world, port, q):
    """One rank of the HIP-backed run: a fresh process (spawned before it makes
    any GPU call), device 0 shared by both ranks.  The rank sizes the whole
    batch on the device (encode_len + scan: the shard plan cuts by encoded
    bytes), encodes and decodes only its own shard with libmhq_huff.so, and
    checks that shard against the oracle; rank 0 checks the gathered whole."""
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        torch.cuda.set_device(0)
        from minhq_amd import hc
        from oracle import oracle

        dev = torch.device("cuda", 0)
        codec = hc.Codec(devices=[0])
        b = workloads.make_batch(20000, "zipf", "hdr", workloads.SEED_ZIPF)
        data = torch.from_numpy(b.data).to(dev)
        off = torch.from_numpy(b.off.view(np.int64).copy()).to(dev)
        n = b.n
        enc_len = torch.empty(n, dtype=torch.int32, device=dev)
        eoff = torch.empty(n + 1, dtype=torch.int64, device=dev)
        cap = torch.empty(n + 1, dtype=torch.int64, device=dev)
        codec.encode_layout_dev(data, off, enc_len, eoff, cap)
        torch.cuda.synchronize()
        lo, hi = shard.plan_shards_device(eoff, world)[rank]
        enc = torch.zeros(int(eoff[-1].item()) + 16, dtype=torch.uint8, device=dev)
        if hi > lo:  # this rank's shard only, in its place in the batch's layout
            codec.encode_dev(data, off[lo:hi + 1], enc, eoff[lo:hi + 1])
        a, c = int(eoff[lo].item()), int(eoff[hi].item())
        s_enc = enc[a:c + 16].clone()
        s_eoff = eoff[lo:hi + 1] - a
        s_cap = cap[lo:hi + 1] - cap[lo]
        out = torch.empty(int(s_cap[-1].item()) + 16, dtype=torch.uint8, device=dev)
        out_len = torch.empty(max(hi - lo, 1), dtype=torch.int32, device=dev)
        status = torch.empty(max(hi - lo, 1), dtype=torch.uint8, device=dev)
        codec.decode_dev(s_enc, s_eoff, out, s_cap, out_len, status)
        torch.cuda.synchronize()
        # the shard against the oracle: its encoding (bytes) and its decode
        e_h, eo_h = s_enc[:c - a].cpu().numpy(), s_eoff.cpu().numpy().view(np.uint64)
        d, o = shard.shard_view(b.data, b.off, lo, hi)
        want_enc = oracle.encode_batch(d, o, eo_h, 1)
        co = s_cap.cpu().numpy().view(np.uint64)
        o_out, o_len, o_st = oracle.decode_batch(e_h, eo_h, co, 1)
        got_out, got_len, got_st = out.cpu().numpy(), out_len.cpu().numpy(), status.cpu().numpy()
        m = hi - lo
        same = (np.array_equal(want_enc, e_h) and np.array_equal(got_len[:m], o_len[:m]) and
                np.array_equal(got_st[:m], o_st[:m]) and
                all(np.array_equal(got_out[int(co[i]):int(co[i]) + int(o_len[i])],
                                   o_out[int(co[i]):int(co[i]) + int(o_len[i])]) for i in range(m)))
        lits = [bytes(got_out[int(co[i]):int(co[i]) + int(got_len[i])]) for i in range(m)]
        gathered = [None] * world
        dist.all_gather_object(gathered, (lo, hi, lits, bool(same)))
        dist.barrier()
        if rank == 0:
            whole = [x for part in sorted(gathered) for x in part[2]]
            want = [bytes(b.data[int(b.off[i]):int(b.off[i + 1])]) for i in range(n)]
            q.put((whole == want, all(p[3] for p in gathered), [p[:2] for p in sorted(gathered)]))
        codec.close()
    finally:
        dist.destroy_process_group()


@pytest.mark.gpu
def test_two_rank_gloo_hip_decode():
    """World size 2 over gloo, both ranks on device 0 through libmhq_huff.so:
    the multi-process path of bench.py's config-4 leg (shard by encoded bytes,
    no data-path collective), every shard compared with the oracle."""
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_hip_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    try:
        ok, shards_ok, ranges = q.get(timeout=240)
    finally:
        for p in procs:
            p.join(timeout=60)
    assert all(p.exitcode == 0 for p in procs)
    assert shards_ok, "a rank's HIP shard differs from the oracle"
    assert ok, "gathered shards differ from the batch"
    assert ranges[0][0] == 0 and ranges[0][1] == ranges[1][0] and ranges[1][1] == 20000
