"""QIF replay with the batch QPACK decoder.

The reference's QIF tool (hc/qif/decoder.go) reads an encoded QIF file as a
sequence of frames, each a 64-bit stream id and a 32-bit length (MSB first,
hc/qif/decoder.go:70-79) followed by that many octets: stream 0 carries
encoder-stream table updates, any other stream one header block.  Decode()
(hc/qif/decoder.go:90-122) feeds them in file order to one QpackDecoder and
writes every block as "name\\tvalue\\n" lines and an empty line
(hc/qif/decoder.go:81-88).

`replay` does the same with QpackBatchDecoder: one host walk over all frames,
one GPU call for every string literal in the file, then the table replay.
"""
from __future__ import annotations

import struct
from typing import Iterable, List, Optional, Tuple

from .headers import HeaderField, QpackBatchDecoder, Reader

QIF_CAPACITY = 4096  # hc.NewQpackDecoder(&devnull, 4096), hc/qif/decoder.go:66


def parse_frames(data: bytes) -> List[Tuple[int, bytes]]:
    """(stream id, payload) frames of an encoded QIF file.  A truncated last
    frame keeps the octets that are there (the LimitedReader's view)."""
    frames, p = [], 0
    while p < len(data):
        if p + 12 > len(data):
            raise EOFError("truncated QIF frame header")
        stream, length = struct.unpack_from(">QI", data, p)
        p += 12
        frames.append((stream, data[p:p + length]))
        p += length
    return frames


def write_frames(frames: Iterable[Tuple[int, bytes]]) -> bytes:
    """The inverse of parse_frames (the framing hc/qif/encoder.go writes)."""
    return b"".join(struct.pack(">QI", s, len(b)) + bytes(b) for s, b in frames)


def format_block(headers: List[HeaderField]) -> bytes:
    """writeBlock (hc/qif/decoder.go:81-88)."""
    return b"".join(h.name + b"\t" + h.value + b"\n" for h in headers) + b"\n"


def replay(data: bytes, capacity: int = QIF_CAPACITY, reader: Optional[Reader] = None):
    """Decodes an encoded QIF file in order.  Returns (text, results): the
    decoder's output text for the header blocks, and per frame the stream id
    with None (updates applied), an Exception, or the header list."""
    frames = parse_frames(data)
    dec = QpackBatchDecoder(capacity, reader)
    res = dec.decode([("updates" if s == 0 else "block", b) for s, b in frames])
    out = []
    for (s, _), r in zip(frames, res):
        if s == 0:
            continue
        if isinstance(r, Exception):
            raise r  # check(err) in hc/qif/decoder.go:117
        out.append(format_block(r))
    return b"".join(out), [(s, r) for (s, _), r in zip(frames, res)]
