"""The in-process multi-device host path (mhq_api.cpp run_host): one context
over several devices splits a host batch into contiguous shards of about equal
encoded bytes (shard_bounds), runs one thread per device (run_shard, each with
its own staging and streams), and writes every shard's results at its own
offsets.  This is the batch analogue of the reference's concurrent block
decode (hc/qif/decoder.go:178-191).

One GPU is enough to run it: mhq_open_devices accepts the same ordinal more
than once, and each entry gets a Device of its own.  Every result is compared
with the oracle (oracle/huff_oracle.c) and with a one-device context.
"""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def lib_built():
    from minhq_amd import build

    build.build()


def _codec(devs):
    from minhq_amd import hc

    return hc.Codec(devices=devs)


def _round_trip(c, oracle_mod, data, off):
    """encode_len / encode / decode through the host ABI on context c, each
    against the oracle; returns the results for cross-context comparison."""
    from minhq_amd import hc

    n = len(off) - 1
    d0 = int(off[0])
    ref_len = oracle_mod.encode_len_batch(np.ascontiguousarray(data), off - np.uint64(d0))
    got_len = c.encode_len(data, off)
    assert np.array_equal(got_len, ref_len)
    enc, enc_off = c.encode(data, off)
    ref_enc = oracle_mod.encode_batch(np.ascontiguousarray(data), off - np.uint64(d0), enc_off)
    assert enc.tobytes() == ref_enc.tobytes()
    cap = hc.capacity_offsets(enc_off)
    out, cap, out_len, st = c.decode(enc, enc_off, cap)
    r_out, r_len, r_st = oracle_mod.decode_batch(np.ascontiguousarray(enc), enc_off, cap)
    assert np.array_equal(out_len, r_len) and np.array_equal(st, r_st)
    for i in range(n):
        a, ln = int(cap[i]), int(out_len[i])
        assert out[a:a + ln].tobytes() == r_out[a:a + ln].tobytes(), i
        assert out[a:a + ln].tobytes() == data[int(off[i]) - d0:int(off[i + 1]) - d0].tobytes(), i
    return got_len, enc, out_len


@pytest.mark.parametrize("devs", [[0, 0], [0, 0, 0, 0]])
def test_uneven_zipf_batch_split_over_devices(lib_built, oracle_mod, devs):
    """Zipf lengths 4..256 (config 4's shape): shards of equal encoded bytes
    hold very different literal counts; the long tail lands in some shards
    only.  Results equal the oracle's and a one-device context's."""
    from minhq_amd import workloads

    b = workloads.make_batch(30000, "zipf", "hdr", workloads.SEED_ZIPF)
    with _codec(devs) as multi, _codec([0]) as single:
        assert multi.ndev == len(devs)
        m = _round_trip(multi, oracle_mod, b.data, b.off)
        s = _round_trip(single, oracle_mod, b.data, b.off)
    for x, y in zip(m, s):
        assert np.array_equal(x, y)


@pytest.mark.parametrize("n", [1, 2, 3])
def test_fewer_literals_than_devices(lib_built, oracle_mod, n):
    """n < D: some shards are empty (run_shard returns at once)."""
    from minhq_amd import hc

    lits = [b"www.example.com", b"", bytes(range(256))][:n]
    data, off = hc.pack(lits)
    with _codec([0, 0, 0, 0]) as c:
        _round_trip(c, oracle_mod, data, off)


def test_biased_offsets_and_garbage_over_devices(lib_built, oracle_mod):
    """A batch whose offsets do not start at 0 (the data pointer is at
    in_off[0]) and a decode of random bytes (INVALID literals, truncating
    garbage) split over two devices, against the oracle."""
    rng = np.random.default_rng(7)
    n = 20000
    lens = rng.integers(0, 60, n)
    off = np.zeros(n + 1, dtype=np.uint64)
    off[1:] = np.cumsum(lens)
    off += np.uint64(12345)  # bias
    data = rng.integers(0x20, 0x7f, int(off[-1] - off[0]), dtype=np.uint8)
    with _codec([0, 0]) as c:
        _round_trip(c, oracle_mod, data, off)
        from minhq_amd import hc

        garbage = rng.integers(0, 256, int(off[-1] - off[0]), dtype=np.uint8)
        garbage[rng.random(len(garbage)) < 0.3] = 0xFF  # EOS prefixes: INVALID literals
        cap = hc.capacity_offsets(off)
        out, cap, out_len, st = c.decode(garbage, off, cap)
        r_out, r_len, r_st = oracle_mod.decode_batch(garbage, off - off[0], cap - cap[0])
        assert np.array_equal(out_len, r_len) and np.array_equal(st, r_st)
        assert (r_st == 1).any()
        for i in range(0, n, 7):
            a, ln = int(cap[i] - cap[0]), int(out_len[i])
            assert out[a:a + ln].tobytes() == r_out[a:a + ln].tobytes(), i
