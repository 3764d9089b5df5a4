"""Pins the CPU oracle (oracle/huff_oracle.c) against the reference's own
known-answer data (tests/golden/, extracted by tests/golden/make_golden.py).

Mirrors hc/huffman_test.go, hc/io_test.go:76-118 and io/bitio_test.go:25-45,
plus the edge cases of the semantics contract.
"""
import random

import pytest


def test_table_matches_reference(oracle_mod, golden):
    lens, vals = oracle_mod.table()
    ref = golden("huffman_table.json")
    assert [r["len"] for r in ref] == lens
    assert [r["val"] for r in ref] == vals


def test_tree_has_513_nodes(oracle_mod):
    # 256 leaves + 256 internal nodes + the childless EOS-prefix node (hc/huffman.go:46-79)
    assert oracle_mod.tree_nodes() == 513


def test_huffman_compress(oracle_mod, golden):  # hc/huffman_test.go:30-46
    for v in golden("huffman_vectors.json"):
        assert oracle_mod.encode(v["text"].encode()).hex() == v["hex"], v["src"]


def test_huffman_decompress(oracle_mod, golden):  # hc/huffman_test.go:48-61
    for v in golden("huffman_vectors.json"):
        out, st = oracle_mod.decode(bytes.fromhex(v["hex"]), cap=len(v["hex"]))
        assert st == oracle_mod.OK
        assert out == v["text"].encode(), v["src"]


def test_embedded_literals(oracle_mod, golden):
    recs = golden("embedded_literals.json")
    texts = {r["text"] for r in recs}
    # the literals SURVEY.md §8c lists must all have been found in the reference's hex
    for t in ["/index.html", "302", "307", "gzip", "name1", "value1", "www.example.com", "no-cache"]:
        assert t in texts
    for r in recs:
        assert oracle_mod.encode(r["text"].encode()).hex() == r["hex"], r["src"]
        out, st = oracle_mod.decode(bytes.fromhex(r["hex"]))
        assert (out, st) == (r["text"].encode(), oracle_mod.OK), r["src"]


def test_read_string(oracle_mod, golden):  # hc/io_test.go:90-101
    for v in golden("string_vectors.json"):
        val, rc, used = oracle_mod.read_string(bytes.fromhex(v["hex"]), v["prefix"])
        assert rc == oracle_mod.OK and val == v["text"].encode(), v["src"]
        assert used == len(v["hex"]) // 2


def test_write_string(oracle_mod, golden):  # hc/io_test.go:103-118
    for v in golden("string_vectors.json"):
        expected = bytes.fromhex(v["hex"])
        choice = 2 if (expected[0] & 0x80) == 0 else 1
        assert oracle_mod.write_string(v["text"].encode(), v["prefix"], choice) == expected, v["src"]


def test_bit_writer(oracle_mod, golden):  # io/bitio_test.go:25-45
    vec = golden("bitio_vectors.json")
    w = oracle_mod.BitWriter()
    for op in vec["ops"]:
        if op["op"] == "bit":
            assert w.write_bit(op["v"]) == 0
        elif op["op"] == "bits":
            assert w.write_bits(op["v"], op["n"]) == 0
        else:
            assert w.pad(op["v"]) == 0
        if op["expect"] is not None:
            assert w.bytes().hex() == op["expect"], op["src"]
    for op in vec["errors"]:  # io/bitio_test.go:90-95
        assert oracle_mod.BitWriter().write_bits(op["v"], op["n"]) == oracle_mod.ERR_TOO_LARGE


# Semantics contract edge cases, derived from hc/huffman.go:46-121.
EDGE = [
    ("", b"", 0),
    ("ff", b"", 0),            # padding only
    ("ffff", b"", 0),
    ("00", b"00"[:1], 0),      # '0' (00000) + 3 zero bits dropped
    ("07", b"0", 0),
    ("3fffffff", b"o", 0),     # 'o' then 26 one bits: partial, dropped
    ("fffffffc", b"", 1),      # 30 ones + more bits: nil child
    ("fffffffd", b"", 1),
    ("ffffffff", b"", 1),
    ("ffffffffff", b"", 1),
]


@pytest.mark.parametrize("hexs,text,st", EDGE)
def test_decode_edge_cases(oracle_mod, hexs, text, st):
    out, got = oracle_mod.decode(bytes.fromhex(hexs))
    assert (out, got) == (text, st)


def test_thirty_ones_at_end_is_accepted(oracle_mod):
    # 'a' (00011) + 30 ones + 1 pad... build 5 + 30 = 35 bits -> 5 bytes with 5 pad bits:
    # the pad makes it 40 bits with 35 ones after 'a' -> more than 30 ones -> invalid.
    # Exactly 30 ones ending the literal: 2 bits of a 2-bit... use 'a'+'a'+30 ones = 40 bits.
    bits = "00011" + "00011" + "1" * 30
    data = int(bits, 2).to_bytes(5, "big")
    out, st = oracle_mod.decode(data)
    assert (out, st) == (b"aa", 0)
    bits = "00011" + "1" * 30 + "0" * 5  # the 31st bit after the ones prefix exists -> invalid
    out, st = oracle_mod.decode(int(bits, 2).to_bytes(5, "big"))
    assert (out, st) == (b"a", 1)


def test_invalid_reports_prefix(oracle_mod):
    enc = oracle_mod.encode(b"abc") + bytes.fromhex("ffffffff")
    out, st = oracle_mod.decode(enc)
    assert st == 1 and out == b"abc"


def test_all_symbols_round_trip(oracle_mod):
    s = bytes(range(256))
    enc = oracle_mod.encode(s)
    assert oracle_mod.decode(enc) == (s, 0)


def test_random_round_trips(oracle_mod):
    rng = random.Random(1234)
    for _ in range(2000):
        s = bytes(rng.randrange(256) for _ in range(rng.randrange(41)))
        enc = oracle_mod.encode(s)
        assert len(enc) == oracle_mod.encoded_len(s)
        assert oracle_mod.decode(enc) == (s, 0)


def test_read_string_edge_cases(oracle_mod):
    # Huffman literal of length 0 -> io.EOF (hc/io.go:92-94 via io.ReadFull)
    assert oracle_mod.read_string(bytes([0x80]))[1] == oracle_mod.ERR_EOF
    # Huffman literal holding only padding -> io.EOF too
    assert oracle_mod.read_string(bytes([0x81, 0xFF]))[1] == oracle_mod.ERR_EOF
    # raw literal of length 0 -> ("", nil)
    assert oracle_mod.read_string(bytes([0x00]))[:2] == (b"", 0)
    # truncated raw literal -> accepted (ErrUnexpectedEOF is success)
    assert oracle_mod.read_string(bytes([0x05]) + b"ab")[:2] == (b"ab", 0)
    # invalid Huffman -> error
    assert oracle_mod.read_string(bytes([0x84, 0xFF, 0xFF, 0xFF, 0xFF]))[1] == oracle_mod.INVALID


def test_auto_choice_is_strictly_shorter(oracle_mod):
    # hc/io.go:172: Auto picks Huffman iff strictly shorter
    for s in [b"a", b"ab", b"www.example.com", b"\x00\x01", b"zzzz"]:
        enc = oracle_mod.encode(s)
        got = oracle_mod.write_string(s, 7, 0)
        if len(enc) < len(s):
            assert got[0] & 0x80 and got[1:] == enc
        else:
            assert not (got[0] & 0x80) and got[1:] == s


def test_batch_drivers_match_single(oracle_mod):
    import numpy as np

    rng = random.Random(7)
    lits = [bytes(rng.randrange(256) for _ in range(rng.randrange(30))) for _ in range(300)]
    off = np.zeros(len(lits) + 1, dtype=np.uint64)
    off[1:] = np.cumsum([len(x) for x in lits])
    data = np.frombuffer(b"".join(lits), dtype=np.uint8).copy()
    enc_len = oracle_mod.encode_len_batch(data, off, nthreads=3)
    assert list(enc_len) == [oracle_mod.encoded_len(x) for x in lits]
    eoff = np.zeros(len(lits) + 1, dtype=np.uint64)
    eoff[1:] = np.cumsum(enc_len)
    enc = oracle_mod.encode_batch(data, off, eoff, nthreads=4)
    assert enc.tobytes() == b"".join(oracle_mod.encode(x) for x in lits)
    cap = np.zeros(len(lits) + 1, dtype=np.uint64)
    cap[1:] = np.cumsum(np.asarray(enc_len, dtype=np.uint64) * 8 // 5)
    out, out_len, status = oracle_mod.decode_batch(enc, eoff, cap, nthreads=2)
    for i, x in enumerate(lits):
        assert out[int(cap[i]): int(cap[i]) + int(out_len[i])].tobytes() == x
    assert not status.any()


def test_netbsd_histogram(golden):
    """workloads.NETBSD_HIST (the `hdr` byte distribution) is the
    byte histogram of the netbsd.qif header set the reference keeps in
    errors.log:7-241 (tests/golden/netbsd_qif.json)."""
    from minhq_amd import workloads

    h = [0] * 95
    for f in golden("netbsd_qif.json")["fields"]:
        for s in f or ():
            for b in s.encode():
                h[b - 0x20] += 1
    assert h == workloads.NETBSD_HIST and sum(h) == 5736


def test_workload_labels():
    from minhq_amd import workloads

    assert workloads.count_label(1 << 24) == "16M" and workloads.count_label(4 << 20) == "4M"
    assert workloads.count_label(1 << 16) == "64K" and workloads.count_label(1000) == "1000"
    assert workloads.config4(1 << 12).name.startswith("config4-4Kx")
    assert workloads.config5(64).name.startswith("config5-64x")


def test_clustered_lengths():
    """The `clustered` length kind (the packed encode's staged-halves timing
    shape, tools/kernel_driver.py clustered:lo:hi): blocks of 512 literals
    alternating U{lo..hi} and U{8..lo}."""
    from minhq_amd import workloads

    L = workloads.lengths("clustered", 4096, 7, 32, 60)
    blocks = L.reshape(8, 512)
    assert all(b.min() >= 32 and b.max() <= 60 for b in blocks[0::2])
    assert all(b.min() >= 8 and b.max() <= 32 for b in blocks[1::2])
    assert 31 < L.mean() < 35


def test_table_driven_decoder_matches_restated(oracle_mod):
    """The table-driven CPU decoder (the honest CPU baseline beside the
    restated Go loop) gives the restated loop's results: valid
    literals, 0xff-heavy garbage (INVALID, partial codes) and truncating
    output regions."""
    import numpy as np

    rng = np.random.default_rng(3)
    lits = [bytes(rng.integers(0, 256, rng.integers(0, 60)).astype(np.uint8)) for _ in range(3000)]
    encs = [oracle_mod.encode(x) for x in lits]
    lens = rng.integers(0, 40, size=3000)
    garb = [bytes(np.where(rng.random(k) < 0.5, 0xFF, rng.integers(0, 256, k)).astype(np.uint8)) for k in lens]
    allb = encs + garb
    off = np.zeros(len(allb) + 1, dtype=np.uint64)
    off[1:] = np.cumsum([len(x) for x in allb])
    data = np.frombuffer(b"".join(allb), dtype=np.uint8).copy()
    for shrink in (0, 3):  # full capacities, then regions 3 bytes short
        caps = np.maximum(np.diff(off) * np.uint64(8) // np.uint64(5), np.uint64(shrink)) - np.uint64(shrink)
        cap = np.zeros(len(off), dtype=np.uint64)
        cap[1:] = np.cumsum(caps)
        o1, l1, s1 = oracle_mod.decode_batch(data, off, cap, nthreads=4)
        o2, l2, s2 = oracle_mod.decode_batch(data, off, cap, nthreads=3, fast=True)
        assert np.array_equal(l1, l2) and np.array_equal(s1, s2) and s1.sum() > 100
        for i in range(len(allb)):
            a = int(cap[i])
            assert o1[a:a + int(l1[i])].tobytes() == o2[a:a + int(l2[i])].tobytes()


@pytest.mark.parametrize("kind,dist,lo,hi,seed", [("uniform", "hdr", 8, 56, 0x6D696E6871),
                                                  ("zipf", "hdr", 8, 56, 0x7A697066),
                                                  ("fixed", "adv", 128, 128, 0x616476),
                                                  ("uniform", "print", 0, 64, 5)])
def test_device_generator_matches_numpy(kind, dist, lo, hi, seed):
    """workloads.make_batch_device (torch, here on the CPU) is bit-identical to
    make_batch (numpy): the full-size bench configs are the same batches."""
    import numpy as np

    from minhq_amd import workloads

    b = workloads.make_batch(3000, kind, dist, seed, lo, hi)
    data, off = workloads.make_batch_device(3000, kind, dist, seed, lo, hi, device="cpu", chunk=1 << 12)
    assert np.array_equal(off.numpy().view(np.uint64), b.off)
    assert np.array_equal(data.numpy(), b.data)
