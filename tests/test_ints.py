"""Prefix integers: batch Reader.ReadInt / ReadIndex and
Writer.WriteInt (hc/io.go:25-67, 110-137).

CPU tests pin the oracle (oracle/huff_oracle.c orc_read_int / orc_write_int)
to the reference's own vectors (hc/io_test.go:11-21 encodedIntegers and
:62-67 TestIntegerOverflow, tests/golden/int_vectors.json); GPU tests run the
read_ints / write_ints kernels through the C ABI and compare them with the
oracle bit-exactly on the same inputs.
"""
import random

import pytest

from oracle import oracle

ORC_EOF, ORC_OVERFLOW = -1, -4
INT_OK, INT_EOF, INT_OVERFLOW = 0, 1, 2


def _vectors(golden):
    g = golden("int_vectors.json")
    return [(int(v["value"]), bytes.fromhex(v["hex"]), v["prefix"], v["src"]) for v in g["ints"]], g["overflow"]


def test_oracle_reads_reference_vectors(golden):  # hc/io_test.go:24-41
    oracle.build()
    ints, _ = _vectors(golden)
    for value, enc, prefix, src in ints:
        v, rc, used = oracle.read_int(enc, prefix, skip_bits=8 - prefix)
        assert (v, rc, used) == (value, 0, len(enc)), src


def test_oracle_writes_reference_vectors(golden):  # hc/io_test.go:43-58
    oracle.build()
    ints, _ = _vectors(golden)
    for value, enc, prefix, src in ints:
        assert oracle.write_int(value, prefix, lead=0, lead_bits=8 - prefix) == enc, src


def test_oracle_overflow_vectors(golden):  # hc/io_test.go:60-75
    oracle.build()
    _, over = _vectors(golden)
    for v in over:
        _, rc, _ = oracle.read_int(bytes.fromhex(v["hex"]), v["prefix"])
        assert rc == ORC_OVERFLOW, v["src"]


def test_oracle_eof_inside_integer():
    oracle.build()
    assert oracle.read_int(b"\x1f\xe1", 5, skip_bits=3)[1] == ORC_EOF  # 4096 cut after one continuation octet
    assert oracle.read_int(b"", 7)[1] == ORC_EOF


def _cases(rng, n):
    """Random integers framed by the oracle's WriteInt with random prefixes and
    opcode bits, plus edge values at every prefix boundary."""
    vals, prefs, leads = [], [], []
    edges = [0, 1, 2, 126, 127, 128, 254, 255, 256, 1 << 14, (1 << 63) - 1, 1 << 63, (1 << 64) - 1]
    for pf in range(1, 9):
        for v in edges + [(1 << pf) - 2, (1 << pf) - 1, (1 << pf)]:
            if v >= 0:
                vals.append(v)
                prefs.append(pf)
                leads.append(rng.randrange(1 << (8 - pf)) if pf < 8 else 0)
    while len(vals) < n:
        pf = rng.randint(1, 8)
        bits = rng.choice([3, 7, 14, 21, 35, 63, 64])
        vals.append(rng.getrandbits(bits))
        prefs.append(pf)
        leads.append(rng.randrange(1 << (8 - pf)) if pf < 8 else 0)
    return vals, prefs, leads


@pytest.fixture(scope="module")
def codec():
    from minhq_amd import build, hc

    build.build()
    c = hc.Codec(1)
    yield c
    c.close()


@pytest.mark.gpu
def test_read_reference_vectors(codec, golden):
    ints, over = _vectors(golden)
    blk, pos, pf, lim = b"", [], [], []
    for value, enc, prefix, _ in ints:
        pos.append(len(blk))
        blk += enc
        lim.append(len(blk))
        pf.append(prefix)
    for v in over:
        pos.append(len(blk))
        blk += bytes.fromhex(v["hex"])
        lim.append(len(blk))
        pf.append(v["prefix"])
    vals, st, nxt = codec.read_ints(blk, pos, pf, lim)
    for i, (value, enc, _, src) in enumerate(ints):
        assert (vals[i], st[i], nxt[i]) == (value, INT_OK, lim[i]), src
    for j, v in enumerate(over):
        i = len(ints) + j
        assert (st[i], nxt[i]) == (INT_OVERFLOW, pos[i]), v["src"]


@pytest.mark.gpu
def test_write_reference_vectors(codec, golden):
    ints, _ = _vectors(golden)
    out = codec.write_ints([v for v, _, _, _ in ints], [p for _, _, p, _ in ints])
    assert out == [enc for _, enc, _, _ in ints]


@pytest.mark.gpu
def test_round_trip_against_oracle(codec):
    rng = random.Random(0x696E74)
    vals, prefs, leads = _cases(rng, 20000)
    frames = codec.write_ints(vals, prefs, leads)
    for v, pf, ld, fr in zip(vals, prefs, leads, frames):
        assert fr == oracle.write_int(v, pf, ld, 8 - pf), (v, pf, ld)
    blk = b"".join(frames)
    pos, lim, p = [], [], 0
    for fr in frames:
        pos.append(p)
        p += len(fr)
        lim.append(p)
    got, st, nxt = codec.read_ints(blk, pos, prefs, lim)
    assert list(st) == [INT_OK] * len(vals)
    assert got == vals and nxt == lim
    # ReadIndex: values above the largest int overflow (hc/io.go:59-67)
    gi, sti, _ = codec.read_ints(blk, pos, prefs, lim, index=True)
    for v, g, s in zip(vals, gi, sti):
        assert (s == INT_OVERFLOW) == (v >> 63 == 1)
        if s == INT_OK:
            assert g == v


@pytest.mark.gpu
def test_truncated_and_garbage_against_oracle(codec):
    rng = random.Random(0x747275)
    vals, prefs, leads = _cases(rng, 4000)
    blk, pos, lim, pf = b"", [], [], []
    for v, p, ld in zip(vals, prefs, leads):
        fr = oracle.write_int(v, p, ld, 8 - p)
        cut = rng.randint(0, len(fr))  # the block ends inside (or right after) the integer
        pos.append(len(blk))
        blk += fr
        lim.append(pos[-1] + cut)
        pf.append(p)
    for _ in range(4000):  # random octets: long runs of continuation bits overflow
        k = rng.randint(1, 14)
        pos.append(len(blk))
        blk += bytes(rng.choice([rng.randrange(256), 0xff, 0x80, 0x81]) for _ in range(k))
        lim.append(len(blk))
        pf.append(rng.randint(1, 8))
    got, st, nxt = codec.read_ints(blk, pos, pf, lim)
    for i in range(len(pos)):
        v, rc, used = oracle.read_int(blk[pos[i]:lim[i]], pf[i], skip_bits=8 - pf[i])
        want = {0: INT_OK, ORC_EOF: INT_EOF, ORC_OVERFLOW: INT_OVERFLOW}[rc]
        assert st[i] == want, i
        if rc == 0:
            assert (got[i], nxt[i]) == (v, pos[i] + used), i
        else:
            assert (got[i], nxt[i]) == (0, pos[i]), i


@pytest.mark.gpu
def test_empty_batches(codec):
    vals, st, nxt = codec.read_ints(b"", [], [])
    assert vals == [] and len(st) == 0 and nxt == []
    assert codec.write_ints([], []) == []
