"""Batch HPACK / QPACK header-block decoding and QIF replay (SURVEY.md §8(f)-2;
minhq_amd/headers.py, minhq_amd/qif.py).

The expected header lists and dynamic tables are the reference's own
(hc/testcases_test.go via tests/golden/header_cases.json), decoded in order
the way hc/hpack_test.go:76-98 (TestHpackDecoder) and hc/qpack_test.go:591-647
(TestQpackDecoderOrdered) do.  CPU tests run the host walk and table replay
with the CPU oracle as the string-literal backend (test infrastructure only);
the GPU tests run the product path, every literal through mhq_read_strings.
"""
import random

import pytest

from minhq_amd import _lib
from minhq_amd.headers import (Blocked, HeaderField, HpackBatchDecoder, IndexError_, PseudoHeaderOrdering,
                               QpackBatchDecoder, TableOverflow)
from minhq_amd import qif
from oracle import oracle

RESET_HPACK = bytes.fromhex("203fe101")  # hc/hpack_test.go:69: capacity 0, then 256


def oracle_reader(blk, pos, prefix, limit):
    """read_strings semantics over the CPU oracle's Reader.ReadString."""
    vals, status, nxt = [], [], []
    for p, pf, lim in zip(pos, prefix, limit):
        val, rc, used = oracle.read_string(blk[p:lim], pf, skip_bits=7 - pf)
        st = {0: _lib.MHQ_STR_OK, 1: _lib.MHQ_STR_INVALID, -1: _lib.MHQ_STR_EOF}[rc]
        vals.append(val if rc == 0 else b"")
        status.append(st)
        nxt.append(p + used)
    return vals, status, nxt


def _hf(h):
    return HeaderField(h["name"].encode(), h["value"].encode(), h["sensitive"])


def _table(entries):
    return [(n.encode(), v.encode()) for n, v in entries]


def run_hpack_cases(cases, reader):
    dec = None
    for i, tc in enumerate(cases):
        if tc["reset"]:
            dec = dec or HpackBatchDecoder(reader)
            assert dec.read_header_blocks([RESET_HPACK]) == [[]]
        got = dec.read_header_blocks([bytes.fromhex(tc["hpack"])])[0]
        assert got == [_hf(h) for h in tc["headers"]], i
        assert dec.table.entries() == _table(tc["hpack_table"]), i
        assert dec.table.used == sum(32 + len(n) + len(v) for n, v in dec.table.entries())


def run_qpack_cases(cases, reader):
    dec = None
    for i, tc in enumerate(cases):
        if tc["reset"]:
            dec = QpackBatchDecoder(256, reader)
        if tc["qpack_updates"]:
            assert dec.read_table_updates(bytes.fromhex(tc["qpack_updates"])) is None, i
            assert dec.table.base == tc["qpack_base"], i
        want_table = tc["qpack_table"] if tc["qpack_table"] is not None else tc["hpack_table"]
        assert dec.table.entries() == _table(want_table), i
        got = dec.read_header_blocks([bytes.fromhex(tc["qpack_header"])])[0]
        assert got == [_hf(h) for h in tc["headers"]], i


def qif_from_cases(cases):
    """One encoded QIF file per reset group: updates on stream 0, header
    blocks on streams 1, 2, ...; and the text Decode() writes for it."""
    files, frames, text, sid = [], [], b"", 0
    for tc in cases:
        if tc["reset"] and frames:
            files.append((qif.write_frames(frames), text))
            frames, text, sid = [], b"", 0
        if tc["qpack_updates"]:
            frames.append((0, bytes.fromhex(tc["qpack_updates"])))
        sid += 1
        frames.append((sid, bytes.fromhex(tc["qpack_header"])))
        text += qif.format_block([_hf(h) for h in tc["headers"]])
    files.append((qif.write_frames(frames), text))
    return files


# ---------------- CPU: walk + replay with the oracle backend ----------------

def test_hpack_reference_cases_cpu(golden):
    oracle.build()
    run_hpack_cases(golden("header_cases.json")["cases"], oracle_reader)


def test_qpack_reference_cases_cpu(golden):
    oracle.build()
    run_qpack_cases(golden("header_cases.json")["cases"], oracle_reader)


def test_qif_replay_cpu(golden):
    oracle.build()
    for data, text in qif_from_cases(golden("header_cases.json")["cases"]):
        got, _ = qif.replay(data, capacity=256, reader=oracle_reader)
        assert got == text


def test_hpack_errors_cpu():
    oracle.build()
    dec = HpackBatchDecoder(oracle_reader)
    res = dec.read_header_blocks([
        bytes([0x90, 0x81]),  # hc/hpack_test.go:101-105: pseudo header after a regular one
        bytes([0xBE]),        # dynamic index 62 into an empty table
        bytes([0xFF, 0x80]),  # index integer cut by the end of the block
        bytes([0x00, 0x84, 0xFF, 0xFF, 0xFF, 0xFC]),  # a Huffman name: 30 ones (EOS prefix) + 2 bits: invalid
        bytes([0x00, 0x81]),  # name length 1, no payload: io.EOF
    ])
    assert isinstance(res[0], PseudoHeaderOrdering)
    assert isinstance(res[1], IndexError_)
    assert isinstance(res[2], EOFError)
    assert isinstance(res[3], ValueError) and "Huffman" in str(res[3])
    assert isinstance(res[4], EOFError)


def test_hpack_eviction_cpu():  # hc/hpack_test.go:107-129 (the decoder half), capacity 64
    oracle.build()
    dec = HpackBatchDecoder(oracle_reader)
    blk = bytes([0x3F, 0x21])  # capacity update to 64
    blk += bytes([0x40, 0x03]) + b"one" + bytes([0x01]) + b"1"
    blk += bytes([0x40, 0x03]) + b"two" + bytes([0x01]) + b"2"
    got = dec.read_header_blocks([blk])[0]
    assert got == [HeaderField(b"one", b"1"), HeaderField(b"two", b"2")]
    assert dec.table.entries() == [(b"two", b"2")]


def test_qpack_errors_cpu():
    oracle.build()
    dec = QpackBatchDecoder(20, oracle_reader)  # hc/qpack_test.go:821-829: one record overflows
    assert isinstance(dec.read_table_updates(bytes.fromhex("4a637573746f6d2d6b65790c637573746f6d2d76616c7565")),
                      TableOverflow)
    dec = QpackBatchDecoder(256, oracle_reader)
    assert isinstance(dec.read_header_blocks([bytes.fromhex("0200c0")])[0], Blocked)  # needs an insert
    assert isinstance(dec.read_header_blocks([bytes.fromhex("0000be")])[0], IndexError_)  # dynamic 62: empty table
    assert isinstance(dec.read_header_blocks([bytes.fromhex("0080")])[0], ValueError)  # sign 1, delta 0


# ---------------- GPU: the product path ----------------

@pytest.mark.gpu
def test_hpack_reference_cases_gpu(golden):
    run_hpack_cases(golden("header_cases.json")["cases"], None)


@pytest.mark.gpu
def test_qpack_reference_cases_gpu(golden):
    run_qpack_cases(golden("header_cases.json")["cases"], None)


@pytest.mark.gpu
def test_qif_replay_gpu(golden):
    for data, text in qif_from_cases(golden("header_cases.json")["cases"]):
        got, _ = qif.replay(data, capacity=256)
        assert got == text


@pytest.mark.gpu
def test_hpack_batch_of_literal_blocks_gpu(golden):
    """netbsd.qif's header set (errors.log:7-241) as HPACK blocks of literals
    without indexing (Huffman chosen by Auto), 2,000 blocks in one batch, vs
    the oracle backend on the same blocks."""
    fields = [(f[0].encode(), f[1].encode()) for f in golden("netbsd_qif.json")["fields"] if f]  # None: block breaks
    rng = random.Random(0x68706B)
    blocks, want = [], []
    for _ in range(2000):
        k = rng.randint(1, 12)
        hs = [fields[rng.randrange(len(fields))] for _ in range(k)]
        hs.sort(key=lambda h: not h[0].startswith(b":"))
        blk = b"".join(bytes([0x00]) + oracle.write_string(n, 7) + oracle.write_string(v, 7) for n, v in hs)
        blocks.append(blk)
        want.append([HeaderField(n, v) for n, v in hs])
    got = HpackBatchDecoder().read_header_blocks(blocks)
    assert got == want
    assert HpackBatchDecoder(oracle_reader).read_header_blocks(blocks) == want
