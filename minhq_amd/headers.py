"""Batch HPACK / QPACK header-block decoding with every string literal decoded
on the GPU in one call.

The reference decodes a header block instruction by instruction, each string
through Reader.ReadString and the bit-serial Huffman tree (hc/hpack.go:68-218,
hc/qpackdecoder.go:126-478).  Here a batch of blocks goes through two passes:

  1. a host walk over the octets of every block locates the instructions: the
     opcodes, their prefix integers and the frame of every string literal (H
     bit and length).  Instruction boundaries never depend on table state or
     on decoded string values, so the walk needs no decoding;
  2. one `read_strings` call decodes all string literals of all blocks on the
     GPU (libmhq_huff.so, `mhq_read_strings`);
  3. a replay applies the dynamic-table semantics in block order with the
     decoded values: inserts, eviction by size, capacity updates, index
     resolution (hc/table.go:100-170, hc/hpack.go:26-52,
     hc/qpacktable.go:35-120), and the reference's error rules.

Results are the reference's per block: the header list, or the error
ReadHeaderBlock returns (ErrIndexError, ErrIntegerOverflow, "invalid Huffman
coding", io.EOF, ErrPseudoHeaderOrdering, ...).  The table state after a
failed block is what the reference leaves: the inserts before the failure.

`reader` is the string-literal backend (blk, pos, prefix, limit) ->
(values, status, next) with MHQ_STR_* statuses; the default is the GPU codec
(minhq_amd.hc.default_codec().read_strings) and nothing else runs in the
product path.
"""
from __future__ import annotations

import json
import os
from dataclasses import dataclass
from typing import Callable, List, Optional, Sequence, Tuple, Union

from . import _lib

HERE = os.path.dirname(os.path.abspath(__file__))
MAX_INT = (1 << 63) - 1
ENTRY_OVERHEAD = 32  # hc/table.go:3, hc/qpacktable.go:7


@dataclass(frozen=True)
class HeaderField:
    """hc.HeaderField (hc/codec.go:13-17)."""

    name: bytes
    value: bytes
    sensitive: bool = False


class IndexError_(LookupError):
    """ErrIndexError: "decoder read an invalid index" (hc/codec.go:10)."""

    def __init__(self):
        super().__init__("decoder read an invalid index")


class PseudoHeaderOrdering(ValueError):
    """ErrPseudoHeaderOrdering (hc/codec.go:12)."""

    def __init__(self):
        super().__init__("invalid pseudo header field order")


class IntegerOverflow(OverflowError):
    """ErrIntegerOverflow (hc/io.go:12)."""

    def __init__(self):
        super().__init__("integer overflow")


class TableOverflow(ValueError):
    """ErrTableOverflow (hc/qpackdecoder.go:132)."""

    def __init__(self):
        super().__init__("table overflow")


class InvalidHuffman(ValueError):
    def __init__(self):
        super().__init__("invalid Huffman coding")


class BlockEOF(EOFError):
    """io.EOF inside an instruction (ReadBits / ReadString)."""

    def __init__(self):
        super().__init__("EOF")


class Blocked(RuntimeError):
    """A QPACK header block needs inserts its updates do not provide
    (QpackDecoderTable.WaitForEntry, hc/qpacktable.go:83-90, would wait)."""


_STATIC = None


def static_tables():
    """HPACK (1-based, 61 entries) and QPACK (0-based) static tables
    (hc/statictable.go), kept as data in static_tables.json."""
    global _STATIC
    if _STATIC is None:
        with open(os.path.join(HERE, "static_tables.json")) as f:
            d = json.load(f)
        _STATIC = {k: [(e["name"].encode(), e["value"].encode()) for e in v] for k, v in d.items()}
    return _STATIC


class DynamicTable:
    """tableCommon (hc/table.go:88-170): newest entry first, absolute base
    counting inserts, eviction from the oldest end by entry size."""

    def __init__(self, capacity: int = 0):
        self.capacity = capacity
        self.used = 0
        self.base = 0
        self.dynamic: List[Tuple[bytes, bytes, int]] = []  # (name, value, base)

    @staticmethod
    def size(name: bytes, value: bytes) -> int:
        return ENTRY_OVERHEAD + len(name) + len(value)

    def get_dynamic(self, i: int, base: int):  # hc/table.go:103-114
        delta = self.base - base
        if delta < 0:
            return None
        j = i + delta
        if j >= len(self.dynamic) or j < 0:
            return None
        return self.dynamic[j]

    def _evict_to(self, reduced: int) -> None:  # hc/table.go:116-129 (no eviction check)
        n, used = len(self.dynamic), self.used
        while n > 0 and used > reduced:
            n -= 1
            used -= self.size(self.dynamic[n][0], self.dynamic[n][1])
        del self.dynamic[n:]
        self.used = used

    def set_capacity(self, capacity: int) -> None:  # hc/table.go:131-134
        self._evict_to(capacity)
        self.capacity = capacity

    def insert(self, name: bytes, value: bytes) -> bool:  # hc/table.go:136-158
        sz = self.size(name, value)
        if sz > self.capacity:
            self.dynamic = []
            self.used = 0
            return False
        self._evict_to(self.capacity - sz)
        self.base += 1
        self.dynamic.insert(0, (name, value, self.base))
        self.used += sz
        return True

    def entries(self) -> List[Tuple[bytes, bytes]]:
        return [(n, v) for n, v, _ in self.dynamic]


# ---- pass 1: the host walk ---------------------------------------------------

class _Walk:
    """Octet cursor over one block (every HPACK/QPACK instruction starts on an
    octet: opcode bits + prefix integer fill the first octet)."""

    def __init__(self, blk: bytes, start: int, end: int, strings: list):
        self.blk, self.p, self.end, self.strings = blk, start, end, strings

    def more(self) -> bool:
        return self.p < self.end

    def top(self) -> int:
        return self.blk[self.p]

    def int_(self, prefix: int, index: bool = False) -> int:
        """Reader.ReadInt / ReadIndex (hc/io.go:25-67) at the current octet."""
        if self.p >= self.end:
            raise BlockEOF()
        mask = (1 << prefix) - 1
        v = self.blk[self.p] & mask
        self.p += 1
        if v == mask:
            s = 0
            while s < 64:
                if self.p >= self.end:
                    raise BlockEOF()
                b = self.blk[self.p]
                self.p += 1
                if s == 63 and (b > 1 or (b == 1 and (v >> 63) == 1)):
                    raise IntegerOverflow()
                v += (b & 0x7F) << s
                if (b & 0x80) == 0:
                    break
                s += 7
        if index and v > MAX_INT:
            raise IntegerOverflow()
        return v

    def string(self, prefix: int) -> int:
        """Frames the string literal at the current octet (H bit and length,
        hc/io.go:73-83) and returns its slot in the batch; the cursor moves past
        the payload, cut at the end of the block like the LimitedReader."""
        slot = len(self.strings)
        self.strings.append((self.p, prefix, self.end))
        if self.p >= self.end:  # ReadBit fails: ("", nil), the cursor stays at EOF
            return slot
        q, mask = self.p, (1 << prefix) - 1
        v = self.blk[q] & mask
        q += 1
        if v == mask:
            s, ok = 0, True
            while s < 64:
                if q >= self.end:
                    ok = False
                    break
                b = self.blk[q]
                q += 1
                if s == 63 and (b > 1 or (b == 1 and (v >> 63) == 1)):
                    ok = False
                    break
                v += (b & 0x7F) << s
                if (b & 0x80) == 0:
                    break
                s += 7
            if not ok:  # ReadInt fails: ("", nil); the reader sits where ReadInt stopped
                self.p = q
                return slot
        self.p = min(q + v, self.end)
        return slot


Op = tuple  # (kind, ...) replayed in pass 2


def _walk_hpack(w: _Walk) -> List[Op]:
    """HpackDecoder.ReadHeaderBlock's instruction walk (hc/hpack.go:147-205)."""
    ops: List[Op] = []
    try:
        while w.more():
            b = w.top()
            if b & 0x80:  # indexed (hc/hpack.go:83-93)
                ops.append(("indexed", w.int_(7, True)))
            elif b & 0x40:  # literal with incremental indexing (hc/hpack.go:95-127)
                idx = w.int_(6, True)
                name = ("str", w.string(7)) if idx == 0 else ("idx", idx)
                ops.append(("incremental", name, w.string(7)))
            elif b & 0x20:  # dynamic table size update (hc/hpack.go:129-136)
                ops.append(("capacity", w.int_(5)))
            else:  # literal without indexing / never indexed (hc/hpack.go:138-148)
                ni = bool(b & 0x10)
                idx = w.int_(4, True)
                name = ("str", w.string(7)) if idx == 0 else ("idx", idx)
                ops.append(("literal", ni, name, w.string(7)))
    except (BlockEOF, IntegerOverflow) as e:
        ops.append(("error", e))
    return ops


def _walk_qpack_updates(w: _Walk) -> List[Op]:
    """QpackDecoder.ReadTableUpdates' walk (hc/qpackdecoder.go:196-236)."""
    ops: List[Op] = []
    try:
        while w.more():
            b = w.top()
            if b & 0x80:  # insert with name reference (hc/qpackdecoder.go:140-160)
                static = bool(b & 0x40)
                idx = w.int_(6, True)
                ops.append(("insert_ref", static, idx, w.string(7)))
            elif b & 0x40:  # insert with name literal (hc/qpackdecoder.go:162-168)
                name = w.string(5)
                ops.append(("insert_lit", name, w.string(7)))
            elif b & 0x20:  # dynamic table size update (hc/qpackdecoder.go:185-193)
                ops.append(("capacity", w.int_(5)))
            else:  # duplicate (hc/qpackdecoder.go:170-183)
                ops.append(("duplicate", w.int_(5, True)))
    except (BlockEOF, IntegerOverflow) as e:
        ops.append(("error", e))
    return ops


def _walk_qpack_block(w: _Walk) -> List[Op]:
    """QpackDecoder.ReadHeaderBlock's walk (hc/qpackdecoder.go:366-478)."""
    ops: List[Op] = []
    try:
        lr_raw = w.int_(8)  # hc/qpackdecoder.go:380
        if not w.more():
            raise BlockEOF()
        sign = bool(w.top() & 0x80)
        delta = w.int_(7, True)  # hc/qpackdecoder.go:389-396
        ops.append(("base", lr_raw, sign, delta))
        while w.more():
            b = w.top()
            if b & 0x80:  # indexed (hc/qpackdecoder.go:240-259)
                ops.append(("indexed", bool(b & 0x40), w.int_(6, True)))
            elif b & 0x40:  # literal with name reference (hc/qpackdecoder.go:276-309)
                ni, static = bool(b & 0x20), bool(b & 0x10)
                idx = w.int_(4, True)
                ops.append(("lit_ref", ni, static, idx, w.string(7)))
            elif b & 0x20:  # literal with name literal (hc/qpackdecoder.go:335-349)
                ni = bool(b & 0x10)
                name = w.string(3)
                ops.append(("lit_lit", ni, name, w.string(7)))
            elif b & 0x10:  # post-base indexed (hc/qpackdecoder.go:261-274)
                ops.append(("post_indexed", w.int_(4, True)))
            else:  # literal with post-base name reference (hc/qpackdecoder.go:311-333)
                ni = bool(b & 0x08)
                idx = w.int_(3, True)
                ops.append(("lit_post", ni, idx, w.string(7)))
    except (BlockEOF, IntegerOverflow) as e:
        ops.append(("error", e))
    return ops


# ---- pass 2: the GPU batch and the replay ------------------------------------

Reader = Callable[[bytes, Sequence[int], Sequence[int], Sequence[int]], tuple]


def _gpu_reader() -> Reader:
    from .hc import default_codec

    return default_codec().read_strings


class _Strings:
    """The decoded string literals of a batch, by slot."""

    def __init__(self, blk: bytes, slots: list, reader: Reader):
        if slots:
            vals, status, _ = reader(blk, [s[0] for s in slots], [s[1] for s in slots], [s[2] for s in slots])
        else:
            vals, status = [], []
        self.vals, self.status = list(vals), [int(x) for x in status]

    def get(self, slot: int) -> bytes:
        st = self.status[slot]
        if st == _lib.MHQ_STR_INVALID:
            raise InvalidHuffman()
        if st == _lib.MHQ_STR_EOF:
            raise BlockEOF()
        if st != _lib.MHQ_STR_OK:
            raise RuntimeError("string literal output buffer too small")
        return self.vals[slot]


Result = Union[List[HeaderField], Exception]


class HpackBatchDecoder:
    """HpackDecoder (hc/hpack.go:68-218) over batches of header blocks, decoded
    in order against one dynamic table."""

    def __init__(self, reader: Optional[Reader] = None):
        self.table = DynamicTable(0)  # new(HpackTable): capacity 0 until an update
        self._reader = reader

    def _get(self, i: int):  # HpackTable.Get (hc/hpack.go:43-52)
        if i <= 0:
            return None
        st = static_tables()["hpack"]
        if i <= len(st):
            return st[i - 1]
        e = self.table.get_dynamic(i - len(st) - 1, self.table.base)
        return None if e is None else (e[0], e[1])

    def _name(self, ref, strings: _Strings) -> bytes:
        if ref[0] == "str":
            return strings.get(ref[1])
        e = self._get(ref[1])
        if e is None:
            raise IndexError_()
        return e[0]

    def read_header_blocks(self, blocks: Sequence[bytes]) -> List[Result]:
        blk = b"".join(blocks)
        slots: list = []
        walks, p = [], 0
        for b in blocks:
            walks.append(_walk_hpack(_Walk(blk, p, p + len(b), slots)))
            p += len(b)
        strings = _Strings(blk, slots, self._reader or _gpu_reader())
        return [self._replay(ops, strings) for ops in walks]

    def _replay(self, ops: List[Op], strings: _Strings) -> Result:
        headers: List[HeaderField] = []
        try:
            for op in ops:
                k = op[0]
                if k == "error":
                    raise op[1]
                if k == "indexed":
                    e = self._get(op[1])
                    if e is None:
                        raise IndexError_()
                    headers.append(HeaderField(e[0], e[1], False))
                elif k == "incremental":
                    name = self._name(op[1], strings)
                    value = strings.get(op[2])
                    self.table.insert(name, value)
                    headers.append(HeaderField(name, value, False))
                elif k == "capacity":
                    self.table.set_capacity(op[1])
                else:  # literal
                    name = self._name(op[2], strings)
                    headers.append(HeaderField(name, strings.get(op[3]), op[1]))
        except Exception as e:  # noqa: BLE001 - the block's error, as ReadHeaderBlock returns it
            return e
        pseudo = True  # hc/hpack.go:207-217
        for h in headers:
            if h.name[:1] == b":":
                if not pseudo:
                    return PseudoHeaderOrdering()
            else:
                pseudo = False
        return headers


class QpackBatchDecoder:
    """QpackDecoder (hc/qpackdecoder.go) over an ordered sequence of
    encoder-stream chunks and header blocks (as hc/qif/decoder.go:90-122 feeds
    them), against one dynamic table of the given capacity."""

    def __init__(self, capacity: int = 256, reader: Optional[Reader] = None):
        self.table = DynamicTable(capacity)
        self._reader = reader

    def _static(self, i: int):  # qpackTableCommon.GetStatic (hc/qpacktable.go:35-44)
        st = static_tables()["qpack"]
        return st[i] if 0 <= i < len(st) else None

    def _dyn(self, i: int, base: int):
        e = self.table.get_dynamic(i, base)
        return None if e is None else (e[0], e[1])

    def _largest_base(self, lr_raw: int) -> int:  # decodeLargestBase (hc/qpackdecoder.go:351-376)
        if lr_raw == 0:
            return 0
        max_entries = self.table.capacity // ENTRY_OVERHEAD
        full = max_entries * 2
        max_value = self.table.base + max_entries
        rounded = max_value // full * full if full else 0
        largest = rounded + lr_raw - 1
        if largest > max_value and largest >= full:
            largest -= full
        return largest

    def decode(self, items: Sequence[Tuple[str, bytes]]) -> List[Optional[Result]]:
        """items: ("updates", bytes) or ("block", bytes), in stream order.
        Returns, per item, None for an update chunk that applied cleanly, the
        error of one that failed, or a header block's result."""
        blk = b"".join(x for _, x in items)
        slots: list = []
        walks, p = [], 0
        for kind, b in items:
            w = _Walk(blk, p, p + len(b), slots)
            walks.append((kind, _walk_qpack_updates(w) if kind == "updates" else _walk_qpack_block(w)))
            p += len(b)
        strings = _Strings(blk, slots, self._reader or _gpu_reader())
        out: List[Optional[Result]] = []
        for kind, ops in walks:
            out.append(self._replay_updates(ops, strings) if kind == "updates" else self._replay_block(ops, strings))
        return out

    def read_table_updates(self, chunk: bytes) -> Optional[Exception]:
        return self.decode([("updates", chunk)])[0]

    def read_header_blocks(self, blocks: Sequence[bytes]) -> List[Result]:
        return self.decode([("block", b) for b in blocks])

    def _insert(self, name: bytes, value: bytes) -> None:  # readValueAndInsert (hc/qpackdecoder.go:126-138)
        if DynamicTable.size(name, value) > self.table.capacity:
            raise TableOverflow()
        self.table.insert(name, value)

    def _replay_updates(self, ops: List[Op], strings: _Strings) -> Optional[Exception]:
        try:
            for op in ops:
                base = self.table.base  # captured per instruction (hc/qpackdecoder.go:201)
                k = op[0]
                if k == "error":
                    raise op[1]
                if k == "insert_ref":
                    e = self._static(op[2]) if op[1] else self._dyn(op[2], base)
                    if e is None:
                        raise IndexError_()
                    self._insert(e[0], strings.get(op[3]))
                elif k == "insert_lit":
                    name = strings.get(op[1])
                    self._insert(name, strings.get(op[2]))
                elif k == "capacity":
                    self.table.set_capacity(op[1])
                else:  # duplicate
                    e = self._dyn(op[1], base)
                    if e is None:
                        raise IndexError_()
                    self.table.insert(e[0], e[1])
        except Exception as e:  # noqa: BLE001
            return e
        return None

    def _replay_block(self, ops: List[Op], strings: _Strings) -> Result:
        headers: List[HeaderField] = []
        try:
            base = 0
            for op in ops:
                k = op[0]
                if k == "error":
                    raise op[1]
                if k == "base":  # readBase (hc/qpackdecoder.go:378-404)
                    largest = self._largest_base(op[1])
                    if self.table.base < largest:
                        raise Blocked(f"header block needs {largest} inserts, table has {self.table.base}")
                    sign, delta = op[2], op[3]
                    if sign and delta == 0:
                        raise ValueError("invalid delta for base index")
                    base = largest + delta * (1 - 2 * int(sign))
                elif k == "indexed":
                    e = self._static(op[2]) if op[1] else self._dyn(op[2], base)
                    if e is None:
                        raise IndexError_()
                    headers.append(HeaderField(e[0], e[1], False))
                elif k == "post_indexed":
                    e = self._dyn(-1 - op[1], base)
                    if e is None:
                        raise IndexError_()
                    headers.append(HeaderField(e[0], e[1], False))
                elif k == "lit_ref":
                    e = self._static(op[3]) if op[2] else self._dyn(op[3], base)
                    if e is None:
                        raise IndexError_()
                    headers.append(HeaderField(e[0], strings.get(op[4]), op[1]))
                elif k == "lit_post":  # GetDynamic(-1*postBase, base) (hc/qpackdecoder.go:323)
                    e = self._dyn(-op[2], base)
                    if e is None:
                        raise IndexError_()
                    headers.append(HeaderField(e[0], strings.get(op[3]), op[1]))
                else:  # lit_lit
                    name = strings.get(op[2])
                    headers.append(HeaderField(name, strings.get(op[3]), op[1]))
        except Exception as e:  # noqa: BLE001
            return e
        return headers
