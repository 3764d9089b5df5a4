"""GPU parity: the HIP kernels (through the C ABI) vs the CPU oracle and the
reference's golden vectors.  Bit-exact throughout (integer/byte work).

Sizes: golden vectors and edge cases; random literals; every BASELINE.json
config at a size the oracle finishes in seconds; and full-size properties
(encode -> decode round trip, out_len == plaintext length) at config sizes.
"""
import random

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


def _oracle_encode_batch(oracle_mod, data, off):
    enc_len = oracle_mod.encode_len_batch(data, off, nthreads=8)
    eoff = np.zeros(len(off), dtype=np.uint64)
    eoff[1:] = np.cumsum(enc_len, dtype=np.uint64)
    return enc_len, oracle_mod.encode_batch(data, off, eoff, nthreads=8), eoff


def _check_batch(codec, oracle_mod, data, off):
    """Encode+decode a packed batch on the GPU; compare with the oracle."""
    from minhq_amd import hc

    enc_len_ref, enc_ref, eoff = _oracle_encode_batch(oracle_mod, data, off)
    assert np.array_equal(codec.encode_len(data, off), enc_len_ref)
    enc, eoff_gpu = codec.encode(data, off)
    assert np.array_equal(eoff_gpu, eoff)
    assert enc.tobytes() == enc_ref.tobytes()
    cap = hc.capacity_offsets(eoff)
    out_ref, len_ref, st_ref = oracle_mod.decode_batch(enc_ref, eoff, cap, nthreads=8)
    out, cap2, out_len, status = codec.decode(enc_ref, eoff, cap)
    assert np.array_equal(out_len, len_ref)
    assert np.array_equal(status, st_ref)
    # compare only the defined bytes of each region
    mask = np.zeros(len(out_ref), dtype=bool)
    starts = cap[:-1].astype(np.int64)
    lens = len_ref.astype(np.int64)
    idx = np.repeat(starts, lens) + (np.arange(lens.sum()) - np.repeat(np.cumsum(lens) - lens, lens))
    mask[idx] = True
    assert np.array_equal(out[: len(out_ref)][mask], out_ref[mask])
    # and the decode reproduces the plaintext
    assert np.array_equal(out_len.astype(np.uint64), np.diff(off))
    assert np.array_equal(out[: len(out_ref)][mask], data)


def test_golden_vectors_batch(codec, golden):
    from minhq_amd import hc

    vecs = golden("huffman_vectors.json") + golden("embedded_literals.json")
    texts = [v["text"].encode() for v in vecs]
    encs = [bytes.fromhex(v["hex"]) for v in vecs]
    assert hc.HuffmanEncodeBatch(texts, codec) == encs
    vals, errs = hc.HuffmanDecodeBatch(encs, codec)
    assert vals == texts and errs == [None] * len(vecs)


EDGE = [
    ("", b"", 0), ("ff", b"", 0), ("ffff", b"", 0), ("00", b"0", 0), ("07", b"0", 0),
    ("3fffffff", b"o", 0), ("fffffffc", b"", 1), ("fffffffd", b"", 1), ("ffffffff", b"", 1),
    ("ffffffffff", b"", 1),
]


def test_edge_cases(codec, oracle_mod):
    from minhq_amd import hc

    encs = [bytes.fromhex(h) for h, _, _ in EDGE]
    # add 30-ones-at-end (accepted) and 31st-bit (invalid) cases, and an invalid tail after text
    encs.append(int("00011" + "00011" + "1" * 30, 2).to_bytes(5, "big"))
    encs.append(int("00011" + "1" * 30 + "0" * 5, 2).to_bytes(5, "big"))
    encs.append(oracle_mod.encode(b"abc") + bytes.fromhex("ffffffff"))
    vals, errs = hc.HuffmanDecodeBatch(encs, codec)
    for e, v, err in zip(encs, vals, errs):
        ref, st = oracle_mod.decode(e)
        assert v == ref, e.hex()
        assert (err is not None) == (st == 1), e.hex()
    assert [v for v in vals[: len(EDGE)]] == [t for _, t, _ in EDGE]


def test_empty_batches(codec, oracle_mod):
    """No literals, and literals that are all empty: the host-buffer entry
    points return empty results without a launch (n == 0) or encode each
    empty literal to zero bytes (HuffmanCompressor.Pad on nothing written,
    hc/huffman.go:30-37) and decode it back to b"" without error."""
    from minhq_amd import hc

    assert hc.HuffmanEncodeBatch([], codec) == []
    assert hc.HuffmanDecodeBatch([], codec) == ([], [])
    lits = [b""] * 1000
    enc = hc.HuffmanEncodeBatch(lits, codec)
    assert enc == [oracle_mod.encode(b"")] * 1000 == [b""] * 1000
    vals, errs = hc.HuffmanDecodeBatch(enc, codec)
    assert vals == lits and errs == [None] * 1000
    # empty literals between non-empty ones keep their slots
    lits = [b"", b"a", b"", b"", b"www.example.com", b""] * 500
    data, off = hc.pack(lits)
    _check_batch(codec, oracle_mod, data, off)


def test_every_symbol_and_long_codes(codec, oracle_mod):
    from minhq_amd import hc

    lits = [bytes(range(256)), bytes(range(255, -1, -1)), bytes([0] * 64), bytes([255] * 64),
            bytes([10, 13, 22] * 40), b"0" * 1000, bytes(range(128, 256)) * 9]
    enc = hc.HuffmanEncodeBatch(lits, codec)
    assert enc == [oracle_mod.encode(x) for x in lits]
    vals, errs = hc.HuffmanDecodeBatch(enc, codec)
    assert vals == lits and errs == [None] * len(lits)


def test_random_bytes_round_trip(codec, oracle_mod):
    rng = random.Random(99)
    lits = [bytes(rng.randrange(256) for _ in range(rng.randrange(0, 90))) for _ in range(5000)]
    from minhq_amd import hc

    data, off = hc.pack(lits)
    _check_batch(codec, oracle_mod, data, off)


def test_encode_len_long_ranges(codec, oracle_mod):
    """encode_len's wave-cooperative path: waves whose byte range takes many
    1-KiB rounds (more than one batch of loads), long literals beside empty
    and one-byte ones, and a wave of short literals next to a long one."""
    rng = random.Random(7)
    sizes = [0, 1, 15, 16, 17, 64, 65, 81, 1000, 5000, 70000, 0, 3, 200000]
    lits = [bytes(rng.randrange(256) for _ in range(k)) for k in sizes]
    lits += [bytes(rng.randrange(32, 127) for _ in range(rng.randrange(0, 60))) for _ in range(300)]
    lits += [bytes(rng.randrange(256) for _ in range(rng.randrange(60, 400))) for _ in range(300)]
    from minhq_amd import hc

    data, off = hc.pack(lits)
    ref = np.array([oracle_mod.encoded_len(x) for x in lits], dtype=np.uint32)
    assert np.array_equal(codec.encode_len(data, off), ref)
    _check_batch(codec, oracle_mod, data, off)


def test_host_round_trip_many_chunks(codec):
    """The host-memory entry points over a batch of many pipelined chunks
    (~37 MB of plaintext, 2 MB chunks on 4 streams; encode_len in 16 MB
    chunks): encode -> decode gives back every literal, and the encoded
    offsets match encode_len's."""
    from minhq_amd import hc, workloads

    b = workloads.config2()
    enc_len = codec.encode_len(b.data, b.off)
    enc, eoff = codec.encode(b.data, b.off)
    assert np.array_equal(np.diff(eoff), enc_len.astype(np.uint64))
    cap = hc.capacity_offsets(eoff)
    out, cap2, out_len, status = codec.decode(enc, eoff, cap)
    assert not status.any()
    assert np.array_equal(out_len.astype(np.uint64), np.diff(b.off))
    starts = cap[:-1].astype(np.int64)
    lens = out_len.astype(np.int64)
    idx = np.repeat(starts - np.cumsum(lens) + lens, lens) + np.arange(int(lens.sum()))
    assert np.array_equal(out[idx], b.data)


def test_random_garbage_decode(codec, oracle_mod):
    """Arbitrary bytes as encoded input: exercises INVALID, partial codes and truncation."""
    from minhq_amd import hc

    rng = np.random.default_rng(5)
    lens = rng.integers(0, 48, size=20000)
    off = np.zeros(len(lens) + 1, dtype=np.uint64)
    off[1:] = np.cumsum(lens)
    # bias toward 0xff so the EOS prefix appears often
    data = np.where(rng.random(int(off[-1])) < 0.5, 0xFF, rng.integers(0, 256, int(off[-1]))).astype(np.uint8)
    cap = hc.capacity_offsets(off)
    out_ref, len_ref, st_ref = oracle_mod.decode_batch(data, off, cap, nthreads=8)
    out, _, out_len, status = codec.decode(data, off, cap)
    assert np.array_equal(out_len, len_ref)
    assert np.array_equal(status, st_ref)
    assert st_ref.sum() > 100  # the INVALID path really is exercised
    for i in range(len(lens)):
        a = int(cap[i])
        assert out[a: a + int(len_ref[i])].tobytes() == out_ref[a: a + int(len_ref[i])].tobytes()


def test_truncating_capacity(codec, oracle_mod):
    """A region smaller than the decoded length is filled and the literal stops OK
    (Read returns once p is full, hc/huffman.go:104)."""
    from minhq_amd import hc

    lits = [b"www.example.com", b"0" * 40, b"custom-value"]
    enc = [oracle_mod.encode(x) for x in lits]
    data, off = hc.pack(enc)
    cap = np.array([0, 4, 4 + 7, 4 + 7 + 100], dtype=np.uint64)
    out, _, out_len, status = codec.decode(data, off, cap)
    for i, e in enumerate(enc):
        c = int(cap[i + 1] - cap[i])
        ref, st = oracle_mod.decode(e, cap=c)
        assert out[int(cap[i]): int(cap[i]) + int(out_len[i])].tobytes() == ref
        assert status[i] == st


def _check_regions(codec, oracle_mod, enc, eoff, cap):
    out, _, out_len, status = codec.decode(enc, eoff, cap)
    ref_out, ref_len, ref_st = oracle_mod.decode_batch(enc, eoff, cap, nthreads=8)
    assert np.array_equal(out_len, ref_len)
    assert np.array_equal(status, ref_st)
    starts = cap[:-1].astype(np.int64)
    lens = ref_len.astype(np.int64)
    idx = np.repeat(starts, lens) + (np.arange(lens.sum()) - np.repeat(np.cumsum(lens) - lens, lens))
    assert np.array_equal(out[idx], ref_out[idx])
    return out, out_len, status


def test_decode_exact_and_short_regions(codec, oracle_mod):
    """Output regions of exactly the plaintext length (a caller that knows the
    lengths, as a round trip does) decode on the fast loop; regions a byte
    short or empty truncate as Read does (hc/huffman.go:104: it returns once p
    is full), as does an INVALID tail behind a region that fills exactly;
    all mixed in one batch, every literal against the oracle."""
    from minhq_amd import workloads

    b = workloads.make_batch(40000, "uniform", "hdr", 11, 0, 64)
    enc_len, enc, eoff = _oracle_encode_batch(oracle_mod, b.data, b.off)
    plain = np.diff(b.off).astype(np.int64)
    # exact regions only: the plaintext comes back
    exact = np.zeros(len(plain) + 1, dtype=np.uint64)
    exact[1:] = np.cumsum(plain)
    out, out_len, status = _check_regions(codec, oracle_mod, enc, eoff, exact)
    assert not status.any() and np.array_equal(out_len.astype(np.int64), plain)
    assert np.array_equal(out[: len(b.data)], b.data)
    # mixed: one byte short, empty, roomy, exact; some literals with 32 one
    # bits after their padding (INVALID, unless their region fills first)
    rng = np.random.default_rng(5)
    kind = rng.integers(0, 8, len(plain))
    lits = [enc[int(eoff[i]): int(eoff[i + 1])].tobytes() for i in range(len(plain))]
    lits = [x + b"\xff\xff\xff\xff" if k == 7 else x for x, k in zip(lits, kind)]
    from minhq_amd import hc
    enc2, eoff2 = hc.pack(lits)
    region = plain.copy()
    region = np.where(kind == 0, np.maximum(plain - 1, 0), region)
    region = np.where(kind == 1, 0, region)
    region = np.where(kind == 2, (np.diff(eoff2).astype(np.int64) * 8) // 5, region)
    cap = np.zeros(len(plain) + 1, dtype=np.uint64)
    cap[1:] = np.cumsum(region)
    _, _, status = _check_regions(codec, oracle_mod, enc2, eoff2, cap)
    assert status[kind == 7].sum() == 0  # their regions fill before the ones are read


@pytest.mark.parametrize("dist", ["hdr", "print", "adv"])
def test_config_batches_vs_oracle(codec, oracle_mod, dist):
    from minhq_amd import workloads

    lo, hi = (128, 128) if dist == "adv" else (8, 64)
    b = workloads.make_batch(20000, "fixed" if dist == "adv" else "uniform", dist, lo=lo, hi=hi)
    _check_batch(codec, oracle_mod, b.data, b.off)


def test_zipf_batch_vs_oracle(codec, oracle_mod):
    from minhq_amd import workloads

    b = workloads.make_batch(30000, "zipf", "hdr", workloads.SEED_ZIPF)
    _check_batch(codec, oracle_mod, b.data, b.off)


def test_qif_corpus_literals(codec, oracle_mod, golden):
    """Config 3: every literal of the netbsd.qif header set (errors.log:7-241) plus
    the reference test-case texts, tiled to 2^16 literals, bit-exact vs the oracle."""
    from minhq_amd import hc

    lits = []
    for f in golden("netbsd_qif.json")["fields"]:
        if f:
            lits += [f[0].encode(), f[1].encode()]
    lits += [r["text"].encode() for r in golden("embedded_literals.json")]
    tiled = (lits * (65536 // len(lits) + 1))[:65536]
    data, off = hc.pack(tiled)
    _check_batch(codec, oracle_mod, data, off)


def test_unaligned_offsets_and_bias(codec, oracle_mod):
    """Host entry points accept offsets that do not start at 0."""
    from minhq_amd import hc

    lits = [b"abc", b"gzip", b"", b"x" * 33]
    enc = [oracle_mod.encode(x) for x in lits]
    data, off = hc.pack(enc)
    off = off + np.uint64(1000)
    cap = hc.capacity_offsets(off) + np.uint64(77)
    out, _, out_len, status = codec.decode(data, off, cap)
    for i, x in enumerate(lits):
        a = int(cap[i] - cap[0])
        assert out[a: a + int(out_len[i])].tobytes() == x


def _device_round_trip(codec, b):
    import torch

    dev = torch.device("cuda:0")
    data = torch.from_numpy(b.data).to(dev)
    off = torch.from_numpy(b.off.view(np.int64)).to(dev)
    n = b.n
    enc_len = torch.empty(n, dtype=torch.int32, device=dev)
    enc_off = torch.empty(n + 1, dtype=torch.int64, device=dev)
    cap_off = torch.empty(n + 1, dtype=torch.int64, device=dev)
    codec.encode_len_dev(data, off, enc_len)
    codec.offsets_dev(enc_len, enc_off, cap_off)
    total = int(enc_off[-1].item())
    enc = torch.empty(max(total, 1), dtype=torch.uint8, device=dev)
    codec.encode_dev(data, off, enc, enc_off)
    out = torch.empty(int(cap_off[-1].item()) + 1, dtype=torch.uint8, device=dev)
    out_len = torch.empty(n, dtype=torch.int32, device=dev)
    status = torch.empty(n, dtype=torch.uint8, device=dev)
    codec.decode_dev(enc, enc_off, out, cap_off, out_len, status)
    torch.cuda.synchronize()
    assert int(status.sum().item()) == 0
    assert torch.equal(out_len.long(), (off[1:] - off[:-1]))
    # gather decoded bytes and compare with the plaintext
    cap = cap_off[:-1]
    lens = out_len.long()
    rep = torch.repeat_interleave(cap, lens)
    within = torch.arange(int(lens.sum().item()), device=dev) - torch.repeat_interleave(
        torch.cumsum(lens, 0) - lens, lens)
    assert torch.equal(out[rep + within], data)
    # capacity_dev on the encoded offsets equals the offsets pass's capacities
    cap2 = torch.empty_like(cap_off)
    codec.capacity_dev(enc_off, cap2)
    torch.cuda.synchronize()
    assert torch.equal(cap2, cap_off)
    # the fused layout call (encode_len + one scan pass) gives the same arrays
    el3 = torch.empty_like(enc_len)
    off3 = torch.empty_like(enc_off)
    cap3 = torch.empty_like(cap_off)
    codec.encode_layout_dev(data, off, el3, off3, cap3)
    torch.cuda.synchronize()
    assert torch.equal(el3, enc_len) and torch.equal(off3, enc_off) and torch.equal(cap3, cap_off)


def test_device_resident_round_trip_full_size(codec):
    """Config 2 at full size (2^20 literals) through the device entry points:
    encode -> offsets -> decode reproduces the plaintext exactly."""
    from minhq_amd import workloads

    _device_round_trip(codec, workloads.config2())


@pytest.mark.parametrize("n", [0, 1, 255, 256, 257, 2047, 2048, 2049, 8 * 2048 + 77, 65535, 65536, 65537,
                               300000, 524287, 524288, 1_100_000, 2_000_000, 4_500_000])
def test_encode_layout_matches_two_pass(codec, n):
    """mhq_huff_encode_layout_dev against encode_len_dev + offsets_dev at the
    block-sum edges (256-literal blocks, 2048-item scan chunks, superblocks
    of 256 sums: 65536 literals for the layout call, 2^19 items for the
    reduce pass), with a base and without cap_off; both against a host scan.
    Up to ~1.45M literals the layout call's apply pass adds up the sums before
    its chunk itself, past that the sums pass runs (offsets_dev: past ~4.2M);
    2M and 4.5M take the three-pass forms."""
    import torch

    from minhq_amd import workloads

    dev = torch.device("cuda:0")
    b = workloads.make_batch(max(n, 1), "uniform", "hdr", lo=0, hi=64)
    data = torch.from_numpy(b.data).to(dev)
    off = torch.from_numpy(b.off.view(np.int64)[: n + 1].copy()).to(dev)
    el1 = torch.full((max(n, 1),), -1, dtype=torch.int32, device=dev)
    o1 = torch.empty(n + 1, dtype=torch.int64, device=dev)
    c1 = torch.empty(n + 1, dtype=torch.int64, device=dev)
    codec.encode_len_dev(data, off, el1)
    codec.offsets_dev(el1[:n], o1, c1, base=12345)
    el2 = torch.full((max(n, 1),), -1, dtype=torch.int32, device=dev)
    o2 = torch.empty(n + 1, dtype=torch.int64, device=dev)
    c2 = torch.empty(n + 1, dtype=torch.int64, device=dev)
    codec.encode_layout_dev(data, off, el2, o2, c2, base=12345)
    o3 = torch.empty(n + 1, dtype=torch.int64, device=dev)
    el3 = torch.empty_like(el2)
    codec.encode_layout_dev(data, off, el3, o3, None, base=12345)
    torch.cuda.synchronize()
    assert torch.equal(el1, el2) and torch.equal(o1, o2) and torch.equal(c1, c2) and torch.equal(o1, o3)
    assert int(o1[0].item()) == 12345
    el = el1[:n].cpu().numpy().astype(np.uint64)
    ref = np.zeros(n + 1, dtype=np.uint64)
    ref[1:] = np.cumsum(el)
    cref = np.zeros(n + 1, dtype=np.uint64)
    cref[1:] = np.cumsum(el * np.uint64(8) // np.uint64(5))
    assert np.array_equal(o1.cpu().numpy().view(np.uint64), ref + np.uint64(12345))
    assert np.array_equal(c1.cpu().numpy().view(np.uint64), cref + np.uint64(12345))


def test_device_resident_round_trip_adversarial_page_aligned(codec):
    """Config 5's literals (128 B of >= 26-bit codes) at 2^20: the plaintext
    buffer ends exactly on a page (and allocation) boundary, so any read
    past the last literal faults."""
    from minhq_amd import workloads

    _device_round_trip(codec, workloads.config5(1 << 20))


def test_encode_empty_region_skips_literal(codec, oracle_mod):
    """mhq_huff_encode_dev: a literal whose output region is empty is skipped
    (nothing written); the others land bit-exactly in their regions.  Covers
    the staged tiles and a literal larger than the staging slice."""
    import torch

    from minhq_amd import hc, workloads

    dev = torch.device("cuda", 0)
    b = workloads.make_batch(5000, "uniform", "hdr", 11, 0, 90)
    lits = hc.unpack(b.data, b.off)
    lits[1234] = bytes(range(256)) * 200  # over the staging slice: the global path
    data, off = hc.pack(lits)
    rng = np.random.default_rng(4)
    keep = rng.random(len(lits)) < 0.6
    keep[1234] = False
    keep[10] = True
    lens = np.array([len(oracle_mod.encode(x)) if k else 0 for x, k in zip(lits, keep)], dtype=np.uint64)
    oo = np.zeros(len(lits) + 1, dtype=np.uint64)
    oo[1:] = np.cumsum(lens)
    out = torch.full((int(oo[-1]) + 16,), 0xAB, dtype=torch.uint8, device=dev)
    codec.encode_dev(torch.from_numpy(data.copy()).to(dev), torch.from_numpy(off.view(np.int64)).to(dev), out,
                     torch.from_numpy(oo.view(np.int64)).to(dev))
    torch.cuda.synchronize()
    got = out.cpu().numpy()
    ref = b"".join(oracle_mod.encode(x) for x, k in zip(lits, keep) if k)
    assert got[: int(oo[-1])].tobytes() == ref
    assert (got[int(oo[-1]):] == 0xAB).all()


def test_host_encode_oversized_regions_gap_bytes(codec, oracle_mod):
    """mhq_huff_encode on pageable buffers (the staged route) into regions
    longer than enc_len, some empty (the literal skipped): the encodings land
    bit-exactly, and every other byte of the copied-back regions is zero --
    never an earlier call's data from the reused device staging buffers
    (the staged encode once skipped zeroing them)."""
    import ctypes as C

    from minhq_amd import hc, workloads

    b = workloads.make_batch(40000, "uniform", "hdr", 12, 8, 64)
    # an earlier call leaves plaintext in the staging buffers
    enc0, eoff0 = codec.encode(b.data, b.off)
    codec.decode(enc0, eoff0)
    lits = hc.unpack(b.data, b.off)
    rng = np.random.default_rng(5)
    enc_len = np.array([len(oracle_mod.encode(x)) for x in lits], dtype=np.uint64)
    keep = rng.random(len(lits)) < 0.9
    extra = rng.integers(0, 24, len(lits)).astype(np.uint64)
    region = np.where(keep, enc_len + extra, 0).astype(np.uint64)
    oo = np.zeros(len(lits) + 1, dtype=np.uint64)
    oo[1:] = np.cumsum(region)
    out = np.full(int(oo[-1]) + 1, 0x5A, dtype=np.uint8)
    data = np.ascontiguousarray(b.data, dtype=np.uint8)
    off = np.ascontiguousarray(b.off, dtype=np.uint64)
    rc = codec._L.mhq_huff_encode(codec.handle, data.ctypes.data_as(C.POINTER(C.c_uint8)),
                                  off.ctypes.data_as(C.POINTER(C.c_uint64)), len(lits),
                                  out.ctypes.data_as(C.POINTER(C.c_uint8)), oo.ctypes.data_as(C.POINTER(C.c_uint64)))
    assert rc == 0
    for i in range(len(lits)):
        a, r = int(oo[i]), int(region[i])
        if not r:
            continue
        e = int(enc_len[i])
        assert out[a:a + e].tobytes() == oracle_mod.encode(lits[i]), i
        assert (out[a + e:a + r] == 0).all(), i
    assert out[-1] == 0x5A


class _Pinned:
    """Allocator of pinned (page-locked) host buffers for the host entry
    points: with every buffer pinned the kernels read and write them in place
    over PCIe (mhq_api.cpp run_zero_copy) instead of staging copies.
    `at_end`: each buffer ends exactly at the end of its pinned block, so an
    input has no slack past it and the call takes the staged path.
    `mhq`: the buffers come from the ABI's own mhq_host_alloc (hc.pinned_empty)
    instead of torch."""

    def __init__(self, at_end=False, mhq=False):
        self.at_end, self.mhq, self.keep = at_end, mhq, []

    def block(self, nbytes):
        if self.mhq:
            from minhq_amd import hc

            return hc.pinned_empty(nbytes)
        import torch

        size = 1 << max(12, (max(nbytes, 1) - 1).bit_length())  # torch's pinned blocks are powers of two
        t = torch.empty(size, dtype=torch.uint8).pin_memory()
        self.keep.append(t)
        a = t.numpy()
        return a[size - nbytes:] if self.at_end else a[:nbytes]

    def __call__(self, nbytes):
        return self.block(nbytes)

    def copy(self, arr):
        arr = np.ascontiguousarray(arr)
        b = self.block(arr.nbytes).view(arr.dtype)
        b[:] = arr
        return b


@pytest.mark.parametrize("source", ["torch", "torch_at_end", "mhq"])
@pytest.mark.parametrize("dist", ["hdr", "adv", "zipf"])
def test_pinned_host_buffers_vs_oracle(codec, oracle_mod, dist, source):
    """Host entry points on pinned buffers (in place over PCIe; staged when
    the inputs end at their block's end) vs the oracle, bit-exact: encode_len,
    encode, decode, including bytes past each out_len left untouched."""
    from minhq_amd import hc, workloads

    if dist == "zipf":
        b = workloads.make_batch(30000, "zipf", "hdr", workloads.SEED_ZIPF)
    else:
        lo, hi = (128, 128) if dist == "adv" else (0, 64)
        b = workloads.make_batch(20000, "fixed" if dist == "adv" else "uniform", dist, lo=lo, hi=hi)
    P = _Pinned(at_end=source == "torch_at_end", mhq=source == "mhq")
    data, off = P.copy(b.data), P.copy(b.off)
    enc_len_ref, enc_ref, eoff = _oracle_encode_batch(oracle_mod, b.data, b.off)
    assert np.array_equal(codec.encode_len(data, off, alloc=P), enc_len_ref)
    enc, eoff_gpu = codec.encode(data, off, alloc=P)
    assert np.array_equal(eoff_gpu, eoff)
    assert enc.tobytes() == enc_ref.tobytes()
    cap = hc.capacity_offsets(eoff)
    out_ref, len_ref, st_ref = oracle_mod.decode_batch(enc_ref, eoff, cap, nthreads=8)
    out, _, out_len, status = codec.decode(P.copy(enc_ref), P.copy(eoff), P.copy(cap), alloc=P)
    assert np.array_equal(out_len, len_ref)
    assert np.array_equal(status, st_ref)
    starts = cap[:-1].astype(np.int64)
    lens = len_ref.astype(np.int64)
    idx = np.repeat(starts, lens) + (np.arange(lens.sum()) - np.repeat(np.cumsum(lens) - lens, lens))
    assert np.array_equal(out[idx], b.data)


def test_pinned_host_garbage_and_bias(codec, oracle_mod):
    """In-place decode of arbitrary bytes (INVALID, truncation) with offsets
    that do not start at 0, against the oracle."""
    from minhq_amd import hc

    rng = np.random.default_rng(11)
    lens = rng.integers(0, 90, 5000)
    off = np.zeros(len(lens) + 1, dtype=np.uint64)
    off[1:] = np.cumsum(lens)
    enc = rng.integers(0, 256, int(off[-1]), dtype=np.uint8)
    cap = hc.capacity_offsets(off)
    out_ref, len_ref, st_ref = oracle_mod.decode_batch(enc, off, cap, nthreads=8)
    P = _Pinned()
    bias, cbias = np.uint64(4093), np.uint64(37)
    out, _, out_len, status = codec.decode(P.copy(enc), P.copy(off + bias), P.copy(cap + cbias), alloc=P)
    assert np.array_equal(out_len, len_ref)
    assert np.array_equal(status, st_ref)
    for i in range(0, len(lens), 7):
        a = int(cap[i])
        assert out[a: a + int(out_len[i])].tobytes() == out_ref[a: a + int(len_ref[i])].tobytes()
