"""The decode's long-literal form (decode_long_kernel, huff_decode.hip): a
batch whose mean literal is over 64 encoded bytes, given its encoded size
(mhq_huff_decode_sized_dev, or the host mhq_huff_decode, which reads it from
its offsets), streams every literal through per-lane windows at 16 waves per
CU.  Against the oracle's Read-to-EOF (hc/huffman.go:102-121) and against the
decode kernel's own results: lengths, statuses, every defined output byte;
long codes only (config 5), long text with INVALID tails, empty literals,
truncating and exact regions.
"""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def codec():
    from minhq_amd import build, hc

    build.build()
    c = hc.Codec(1)
    yield c
    c.close()


def _dev_decode(codec, enc, eoff, cap, in_bytes):
    import torch

    dev = torch.device("cuda:0")
    n = len(eoff) - 1
    t_enc = torch.from_numpy(np.ascontiguousarray(enc, dtype=np.uint8).copy() if len(enc) else np.zeros(1, np.uint8)).to(dev)
    t_off = torch.from_numpy(eoff.astype(np.uint64).view(np.int64).copy()).to(dev)
    t_cap = torch.from_numpy(cap.astype(np.uint64).view(np.int64).copy()).to(dev)
    out = torch.full((int(cap[-1]) + 1,), 0xA5, dtype=torch.uint8, device=dev)
    out_len = torch.full((max(n, 1),), -1, dtype=torch.int32, device=dev)
    status = torch.full((max(n, 1),), 0x77, dtype=torch.uint8, device=dev)
    torch.cuda.synchronize()
    codec.decode_dev(t_enc, t_off, out, t_cap, out_len, status, in_bytes=in_bytes)
    torch.cuda.synchronize()
    return out.cpu().numpy(), out_len.cpu().numpy()[:n].view(np.uint32), status.cpu().numpy()[:n]


def _check(codec, oracle_mod, enc, eoff, cap):
    ref_out, ref_len, ref_st = oracle_mod.decode_batch(enc, eoff, cap, nthreads=8)
    in_bytes = int(eoff[-1] - eoff[0])
    assert in_bytes > 64 * (len(eoff) - 1), "not a long-literal batch"
    got = {}
    for name, ib in (("long", in_bytes), ("tiles", 0)):
        out, out_len, status = _dev_decode(codec, enc, eoff, cap, ib)
        assert np.array_equal(out_len, ref_len), name
        assert np.array_equal(status, ref_st), name
        starts = cap[:-1].astype(np.int64)
        lens = ref_len.astype(np.int64)
        idx = np.repeat(starts, lens) + (np.arange(lens.sum()) - np.repeat(np.cumsum(lens) - lens, lens))
        assert np.array_equal(out[idx], ref_out[idx]), name
        got[name] = (out_len, status)
    return ref_len, ref_st


def test_long_codes_config5(codec, oracle_mod):
    """Config 5's shape: 128-byte literals of bytes whose codes are >= 26 bits."""
    from minhq_amd import hc, workloads as w

    b = w.config5(6000)
    enc_len = oracle_mod.encode_len_batch(b.data, b.off, nthreads=8)
    eoff = np.zeros(b.n + 1, dtype=np.uint64)
    eoff[1:] = np.cumsum(enc_len, dtype=np.uint64)
    enc = oracle_mod.encode_batch(b.data, b.off, eoff, nthreads=8)
    ref_len, ref_st = _check(codec, oracle_mod, enc, eoff, hc.capacity_offsets(eoff))
    assert np.array_equal(ref_len.astype(np.uint64), np.diff(b.off)) and not ref_st.any()


def test_long_text_invalid_empty_and_regions(codec, oracle_mod):
    """Long text literals (70-600 B), some with 32 one bits past their padding
    (INVALID), some with random tails, empty ones; regions roomy, exact, a
    byte short and empty."""
    from minhq_amd import hc

    rng = np.random.default_rng(71)
    n = 9000
    lits, plain = [], []
    for i in range(n):
        k = int(rng.integers(0, 10))
        if k == 0:
            lits.append(b"")
            plain.append(0)
            continue
        t = bytes(rng.integers(32, 127, int(rng.integers(90, 800)), dtype=np.uint8))
        e = oracle_mod.encode(t)
        if k == 1:
            e += b"\xff\xff\xff\xff"
        elif k == 2:
            e += bytes(rng.integers(0, 256, 5, dtype=np.uint8))
        lits.append(e)
        plain.append(len(t))
    enc, eoff = hc.pack(lits)
    cap_roomy = hc.capacity_offsets(eoff)
    _check(codec, oracle_mod, enc, eoff, cap_roomy)
    plain = np.array(plain, dtype=np.int64)
    kind = rng.integers(0, 4, n)
    region = np.where(kind == 0, plain, np.where(kind == 1, np.maximum(plain - 1, 0),
                                                 np.where(kind == 2, 0, (np.diff(eoff).astype(np.int64) * 8) // 5)))
    cap = np.zeros(n + 1, dtype=np.uint64)
    cap[1:] = np.cumsum(region)
    _check(codec, oracle_mod, enc, eoff, cap)


def test_long_host_path(codec, oracle_mod):
    """The host-memory decode picks the long form from its own offsets."""
    from minhq_amd import hc

    rng = np.random.default_rng(72)
    lits = [oracle_mod.encode(bytes(rng.integers(0, 256, int(rng.integers(40, 200)), dtype=np.uint8)))
            for _ in range(3000)]
    enc, eoff = hc.pack(lits)
    assert int(eoff[-1]) > 64 * 3000
    cap = hc.capacity_offsets(eoff)
    ref_out, ref_len, ref_st = oracle_mod.decode_batch(enc, eoff, cap, nthreads=8)
    out, _, out_len, status = codec.decode(enc, eoff, cap)
    assert np.array_equal(out_len, ref_len) and np.array_equal(status, ref_st)
    for i in range(len(lits)):
        a = int(cap[i])
        assert out[a: a + int(ref_len[i])].tobytes() == ref_out[a: a + int(ref_len[i])].tobytes()
