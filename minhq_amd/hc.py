"""Host-side mirror of minhq's `hc` Huffman surface over the HIP C ABI.

The reference's streaming API (hc/huffman.go:11-121) is one literal at a time
and stays in Go; what this build adds behind it is the batch path that the
cgo shim in INTEGRATION.md exposes as

    hc.HuffmanEncodeBatch(lits [][]byte) [][]byte
    hc.HuffmanDecodeBatch(enc  [][]byte) ([][]byte, []error)

This module is that shim's Python twin (ctypes instead of cgo), so the parity
tests drive the library exactly as Go would: pack literals into one byte
buffer plus uint64 offsets, call the C ABI, unpack.  Names, argument meaning
and error behaviour follow the reference:

* HuffmanEncodeBatch(lits)[i] == Write(lits[i]) + Pad()   (hc/huffman.go:23-37)
* HuffmanDecodeBatch(enc)[i]  == Read to EOF of enc[i]    (hc/huffman.go:102-121);
  an invalid code gives the bytes produced so far and
  InvalidHuffmanCoding("invalid Huffman coding") (hc/huffman.go:112).
* HuffmanCodingAuto/Always/Never and the strictly-shorter Auto rule
  (hc/io.go:140-150, :172) are exposed for callers that frame literals.

There is no CPU fallback: every entry point runs on the gfx950 library and
raises if it cannot.
"""
from __future__ import annotations

import ctypes as C
from typing import List, Optional, Sequence, Tuple

import numpy as np

from . import _lib
from ._lib import MhqError, check

# hc/io.go:140-150
HuffmanCodingAuto = 0
HuffmanCodingAlways = 1
HuffmanCodingNever = 2


class InvalidHuffmanCoding(ValueError):
    """errors.New("invalid Huffman coding") -- hc/huffman.go:112."""

    def __init__(self):
        super().__init__("invalid Huffman coding")


def pack(lits: Sequence[bytes]) -> Tuple[np.ndarray, np.ndarray]:
    """Packs literals back to back; returns (bytes u8[], offsets u64[n+1])."""
    off = np.zeros(len(lits) + 1, dtype=np.uint64)
    if lits:
        off[1:] = np.cumsum([len(x) for x in lits], dtype=np.uint64)
    data = np.frombuffer(b"".join(lits), dtype=np.uint8) if lits else np.zeros(0, np.uint8)
    return np.ascontiguousarray(data), off


def unpack(data: np.ndarray, off: np.ndarray, lens: Optional[np.ndarray] = None) -> List[bytes]:
    buf = data.tobytes()
    base = int(off[0]) if len(off) else 0
    out = []
    for i in range(len(off) - 1):
        a = int(off[i]) - base
        b = a + int(lens[i]) if lens is not None else int(off[i + 1]) - base
        out.append(buf[a:b])
    return out


def capacity_offsets(enc_off: np.ndarray) -> np.ndarray:
    """cap_off for decode: floor(8*len/5) per literal (hc/io.go:87 allocates one more)."""
    lens = np.diff(enc_off.astype(np.uint64))
    cap = np.zeros(len(enc_off), dtype=np.uint64)
    if len(lens):
        cap[1:] = np.cumsum(lens * np.uint64(8) // np.uint64(5), dtype=np.uint64)
    return cap


def _p(a: np.ndarray, t):
    return a.ctypes.data_as(C.POINTER(t))


def pinned_empty(nbytes: int) -> np.ndarray:
    """A uint8 array in pinned, device-mapped host memory (mhq_host_alloc):
    host-memory calls whose buffers are all such arrays run in place (the
    kernels read and write them over PCIe).  Freed with the
    array."""
    import weakref

    L = _lib.load()
    n = max(int(nbytes), 1)
    p = L.mhq_host_alloc(n)
    if not p:
        raise MemoryError(f"mhq_host_alloc({n}) failed")
    buf = (C.c_uint8 * n).from_address(p)
    weakref.finalize(buf, L.mhq_host_free, p)
    return np.frombuffer(buf, dtype=np.uint8)[: int(nbytes)]


def pinned_copy(a: np.ndarray) -> np.ndarray:
    """`a` copied into pinned_empty memory (same dtype and shape)."""
    a = np.ascontiguousarray(a)
    out = pinned_empty(a.nbytes).view(a.dtype).reshape(a.shape)
    out[...] = a
    return out


class PinnedAllocator:
    """`alloc=` for the Codec's host-memory methods: every output in pinned
    memory (pinned_empty), so with pinned inputs the call runs in place."""

    def __call__(self, nbytes: int) -> np.ndarray:
        return pinned_empty(nbytes)


def _alloc(alloc, n: int, dtype) -> np.ndarray:
    if alloc is None:
        return np.zeros(n, dtype=dtype)
    return alloc(n * np.dtype(dtype).itemsize)[: n * np.dtype(dtype).itemsize].view(dtype)


def _nonempty(a: np.ndarray) -> np.ndarray:
    # ctypes needs a valid pointer even for zero-length buffers
    return a if a.size else np.zeros(1, dtype=a.dtype)


class Codec:
    """An mhq_ctx: the device tables and staging buffers on `ndev` GPUs (0 = all),
    or on the explicit HIP device ordinals `devices`."""

    def __init__(self, ndev: int = 0, devices: Optional[Sequence[int]] = None):
        self._L = _lib.load()
        h = C.c_void_p()
        if devices is not None:
            arr = (C.c_int * len(devices))(*devices)
            check(self._L.mhq_open_devices(C.byref(h), arr, len(devices)), "mhq_open_devices")
        else:
            check(self._L.mhq_open(C.byref(h), ndev), "mhq_open")
        self._h = h

    @property
    def handle(self):
        return self._h

    @property
    def ndev(self) -> int:
        return self._L.mhq_device_count(self._h)

    def close(self) -> None:
        if getattr(self, "_h", None):
            self._L.mhq_close(self._h)
            self._h = None

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        self.close()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    # ---------------- host-memory batches ----------------
    # `alloc(nbytes) -> uint8 array` supplies the output buffers of the
    # host-memory calls (e.g. pinned memory for the PCIe-inclusive rate); the
    # default is zeroed pageable numpy memory.
    def encode_len(self, data: np.ndarray, off: np.ndarray, alloc=None) -> np.ndarray:
        n = len(off) - 1
        out = _alloc(alloc, max(n, 1), np.uint32)
        data = _nonempty(np.ascontiguousarray(data, dtype=np.uint8))
        off = np.ascontiguousarray(off, dtype=np.uint64)
        check(self._L.mhq_huff_encode_len(self._h, _p(data, C.c_uint8), _p(off, C.c_uint64), n,
                                          _p(out, C.c_uint32)), "mhq_huff_encode_len")
        return out[:n]

    def encode(self, data: np.ndarray, off: np.ndarray, alloc=None) -> Tuple[np.ndarray, np.ndarray]:
        """Returns (encoded bytes, encoded offsets) for a packed batch."""
        n = len(off) - 1
        # enc_len from the caller's allocator too: in pinned memory the kernel
        # writes it in place (the host scan reads pinned memory as fast as
        # pageable: 0.34 vs 0.36 ms for 2^20 lengths, tools/hostpath.py)
        enc_len = self.encode_len(data, off, alloc=alloc)
        enc_off = _alloc(alloc, n + 1, np.uint64)
        enc_off[0] = 0
        if n:
            enc_off[1:] = np.cumsum(enc_len, dtype=np.uint64)
        out = _alloc(alloc, max(int(enc_off[-1]), 1), np.uint8)
        data = _nonempty(np.ascontiguousarray(data, dtype=np.uint8))
        off = np.ascontiguousarray(off, dtype=np.uint64)
        check(self._L.mhq_huff_encode(self._h, _p(data, C.c_uint8), _p(off, C.c_uint64), n,
                                      _p(out, C.c_uint8), _p(enc_off, C.c_uint64)), "mhq_huff_encode")
        return out[: int(enc_off[-1])], enc_off

    def decode(self, enc: np.ndarray, off: np.ndarray, cap_off: Optional[np.ndarray] = None, alloc=None):
        """Returns (out, cap_off, out_len, status) for a packed batch."""
        n = len(off) - 1
        off = np.ascontiguousarray(off, dtype=np.uint64)
        if cap_off is None:
            cap_off = capacity_offsets(off)
        cap_off = np.ascontiguousarray(cap_off, dtype=np.uint64)
        out = _alloc(alloc, max(int(cap_off[-1] - cap_off[0]) if n else 0, 1), np.uint8)
        out_len = _alloc(alloc, max(n, 1), np.uint32)
        status = _alloc(alloc, max(n, 1), np.uint8)
        enc = _nonempty(np.ascontiguousarray(enc, dtype=np.uint8))
        check(self._L.mhq_huff_decode(self._h, _p(enc, C.c_uint8), _p(off, C.c_uint64), n,
                                      _p(out, C.c_uint8), _p(cap_off, C.c_uint64), _p(out_len, C.c_uint32),
                                      _p(status, C.c_uint8)), "mhq_huff_decode")
        return out, cap_off, out_len[:n], status[:n]

    # ---------------- string literals (hc/io.go:73-97, 153-197) ---------------
    def read_strings(self, blk: bytes, pos: Sequence[int], prefix: Sequence[int],
                     limit: Optional[Sequence[int]] = None):
        """Batch Reader.ReadString: literal i at byte pos[i] (H bit = bit 7-prefix[i])
        reading up to limit[i] (default: the end of blk).  Returns
        (values, status, next) with status MHQ_STR_* per literal."""
        n = len(pos)
        blk_a = _nonempty(np.frombuffer(bytes(blk), dtype=np.uint8).copy())
        pos_a = _nonempty(np.ascontiguousarray(pos, dtype=np.uint64))
        lim_a = _nonempty(np.ascontiguousarray(limit if limit is not None else [len(blk)] * n, dtype=np.uint64))
        pf_a = _nonempty(np.ascontiguousarray(prefix, dtype=np.uint8))
        cap = len(blk) * 8 // 5 + 16
        out = np.zeros(cap, dtype=np.uint8)
        out_off = np.zeros(n + 1, dtype=np.uint64)
        out_len = np.zeros(max(n, 1), dtype=np.uint32)
        status = np.zeros(max(n, 1), dtype=np.uint8)
        nxt = np.zeros(max(n, 1), dtype=np.uint64)
        check(self._L.mhq_read_strings(self._h, _p(blk_a, C.c_uint8), len(blk), _p(pos_a, C.c_uint64),
                                       _p(lim_a, C.c_uint64), _p(pf_a, C.c_uint8), n, _p(out, C.c_uint8), cap,
                                       _p(out_off, C.c_uint64), _p(out_len, C.c_uint32), _p(status, C.c_uint8),
                                       _p(nxt, C.c_uint64)), "mhq_read_strings")
        vals = [out[int(out_off[i]): int(out_off[i]) + int(out_len[i])].tobytes() for i in range(n)]
        return vals, status[:n].copy(), nxt[:n].copy()

    def write_strings(self, strs: Sequence[bytes], prefix: Sequence[int], lead: Optional[Sequence[int]] = None,
                      choice: int = HuffmanCodingAuto) -> List[bytes]:
        """Batch Writer.WriteStringRaw(s, prefix, choice) after opcode bits lead[i]."""
        n = len(strs)
        data, off = pack(strs)
        data = _nonempty(data)
        pf_a = _nonempty(np.ascontiguousarray(prefix, dtype=np.uint8))
        ld_a = _nonempty(np.ascontiguousarray(lead if lead is not None else [0] * n, dtype=np.uint8))
        out_off = np.zeros(n + 1, dtype=np.uint64)
        check(self._L.mhq_write_strings(self._h, _p(data, C.c_uint8), _p(off, C.c_uint64), n, _p(pf_a, C.c_uint8),
                                        _p(ld_a, C.c_uint8), choice, None, 0, _p(out_off, C.c_uint64), None),
              "mhq_write_strings (size)")
        cap = int(out_off[-1]) if n else 0
        out = np.zeros(max(cap, 1), dtype=np.uint8)
        status = np.zeros(max(n, 1), dtype=np.uint8)
        check(self._L.mhq_write_strings(self._h, _p(data, C.c_uint8), _p(off, C.c_uint64), n, _p(pf_a, C.c_uint8),
                                        _p(ld_a, C.c_uint8), choice, _p(out, C.c_uint8), cap,
                                        _p(out_off, C.c_uint64), _p(status, C.c_uint8)), "mhq_write_strings")
        if n and np.any(status[:n] != _lib.MHQ_STR_OK):
            raise RuntimeError("mhq_write_strings: output buffer too small")
        return unpack(out, out_off)

    # ---------------- prefix integers (hc/io.go:25-67, 110-137) ---------------
    def read_ints(self, blk: bytes, pos: Sequence[int], prefix: Sequence[int],
                  limit: Optional[Sequence[int]] = None, index: bool = False):
        """Batch Reader.ReadInt (ReadIndex with index=True): integer i at byte
        pos[i], its prefix in the low prefix[i] bits, reading up to limit[i]
        (default: the end of blk).  Returns (values, status, next) with
        status MHQ_INT_* per integer."""
        n = len(pos)
        blk_a = _nonempty(np.frombuffer(bytes(blk), dtype=np.uint8).copy())
        pos_a = _nonempty(np.ascontiguousarray(pos, dtype=np.uint64))
        lim_a = _nonempty(np.ascontiguousarray(limit if limit is not None else [len(blk)] * n, dtype=np.uint64))
        pf_a = _nonempty(np.ascontiguousarray(prefix, dtype=np.uint8))
        val = np.zeros(max(n, 1), dtype=np.uint64)
        nxt = np.zeros(max(n, 1), dtype=np.uint64)
        status = np.zeros(max(n, 1), dtype=np.uint8)
        check(self._L.mhq_read_ints(self._h, _p(blk_a, C.c_uint8), len(blk), _p(pos_a, C.c_uint64),
                                    _p(lim_a, C.c_uint64), _p(pf_a, C.c_uint8), n, 1 if index else 0,
                                    _p(val, C.c_uint64), _p(nxt, C.c_uint64), _p(status, C.c_uint8)),
              "mhq_read_ints")
        return [int(v) for v in val[:n]], status[:n].copy(), [int(x) for x in nxt[:n]]

    def write_ints(self, values: Sequence[int], prefix: Sequence[int],
                   lead: Optional[Sequence[int]] = None) -> List[bytes]:
        """Batch Writer.WriteInt(v, prefix) after opcode bits lead[i]."""
        n = len(values)
        val_a = _nonempty(np.array([int(v) for v in values], dtype=np.uint64))
        pf_a = _nonempty(np.ascontiguousarray(prefix, dtype=np.uint8))
        ld_a = _nonempty(np.ascontiguousarray(lead if lead is not None else [0] * n, dtype=np.uint8))
        out_off = np.zeros(n + 1, dtype=np.uint64)
        check(self._L.mhq_write_ints(self._h, _p(val_a, C.c_uint64), _p(pf_a, C.c_uint8), _p(ld_a, C.c_uint8), n,
                                     None, 0, _p(out_off, C.c_uint64), None), "mhq_write_ints (size)")
        cap = int(out_off[-1]) if n else 0
        out = np.zeros(max(cap, 1), dtype=np.uint8)
        status = np.zeros(max(n, 1), dtype=np.uint8)
        check(self._L.mhq_write_ints(self._h, _p(val_a, C.c_uint64), _p(pf_a, C.c_uint8), _p(ld_a, C.c_uint8), n,
                                     _p(out, C.c_uint8), cap, _p(out_off, C.c_uint64), _p(status, C.c_uint8)),
              "mhq_write_ints")
        if n and np.any(status[:n] != _lib.MHQ_INT_OK):
            raise ValueError("mhq_write_ints: prefix outside 1..8")
        return unpack(out, out_off)

    # ---------------- HTTP/3 (draft) frame varints (frame.go:72-92, 128-152) --
    def _blk_args(self, blk, pos, limit):
        n = len(pos)
        blk_a = _nonempty(np.frombuffer(bytes(blk), dtype=np.uint8).copy())
        pos_a = _nonempty(np.ascontiguousarray(pos, dtype=np.uint64))
        lim_a = _nonempty(np.ascontiguousarray(limit if limit is not None else [len(blk)] * n, dtype=np.uint64))
        return n, blk_a, pos_a, lim_a

    def read_varints(self, blk: bytes, pos: Sequence[int], limit: Optional[Sequence[int]] = None):
        """Batch frameReader.ReadVarint: (values, status, next), status MHQ_VARINT_*."""
        n, blk_a, pos_a, lim_a = self._blk_args(blk, pos, limit)
        val = np.zeros(max(n, 1), dtype=np.uint64)
        nxt = np.zeros(max(n, 1), dtype=np.uint64)
        st = np.zeros(max(n, 1), dtype=np.uint8)
        check(self._L.mhq_read_varints(self._h, _p(blk_a, C.c_uint8), len(blk), _p(pos_a, C.c_uint64),
                                       _p(lim_a, C.c_uint64), n, _p(val, C.c_uint64), _p(nxt, C.c_uint64),
                                       _p(st, C.c_uint8)), "mhq_read_varints")
        return [int(v) for v in val[:n]], st[:n].copy(), [int(x) for x in nxt[:n]]

    def read_frames(self, blk: bytes, pos: Sequence[int], limit: Optional[Sequence[int]] = None):
        """Batch ReadFrame headers: (types, payload lengths, payload positions, status)."""
        n, blk_a, pos_a, lim_a = self._blk_args(blk, pos, limit)
        typ = np.zeros(max(n, 1), dtype=np.uint8)
        plen = np.zeros(max(n, 1), dtype=np.uint64)
        ppos = np.zeros(max(n, 1), dtype=np.uint64)
        st = np.zeros(max(n, 1), dtype=np.uint8)
        check(self._L.mhq_read_frames(self._h, _p(blk_a, C.c_uint8), len(blk), _p(pos_a, C.c_uint64),
                                      _p(lim_a, C.c_uint64), n, _p(typ, C.c_uint8), _p(plen, C.c_uint64),
                                      _p(ppos, C.c_uint64), _p(st, C.c_uint8)), "mhq_read_frames")
        return ([int(t) for t in typ[:n]], [int(x) for x in plen[:n]], [int(x) for x in ppos[:n]],
                st[:n].copy())

    def write_varints(self, values: Sequence[int]):
        """Batch frameWriter.WriteVarint: (encodings, status); a value >= 2^62
        gives b"" and MHQ_VARINT_TOO_LARGE (ErrTooLarge)."""
        n = len(values)
        val_a = _nonempty(np.array([int(v) for v in values], dtype=np.uint64))
        out_off = np.zeros(n + 1, dtype=np.uint64)
        check(self._L.mhq_write_varints(self._h, _p(val_a, C.c_uint64), n, None, 0, _p(out_off, C.c_uint64), None),
              "mhq_write_varints (size)")
        cap = int(out_off[-1]) if n else 0
        out = np.zeros(max(cap, 1), dtype=np.uint8)
        st = np.zeros(max(n, 1), dtype=np.uint8)
        check(self._L.mhq_write_varints(self._h, _p(val_a, C.c_uint64), n, _p(out, C.c_uint8), cap,
                                        _p(out_off, C.c_uint64), _p(st, C.c_uint8)), "mhq_write_varints")
        return unpack(out, out_off), st[:n].copy()

    # ---------------- device-resident batches (torch tensors on one device) ---
    @staticmethod
    def _stream(stream):
        if stream is None:
            import torch

            return C.c_void_p(torch.cuda.current_stream().cuda_stream)
        return C.c_void_p(int(stream))

    def encode_len_dev(self, data, off, enc_len, dev: int = 0, stream=None) -> None:
        n = off.numel() - 1
        check(self._L.mhq_huff_encode_len_dev(self._h, dev, data.data_ptr(), off.data_ptr(), n,
                                              enc_len.data_ptr(), self._stream(stream)), "encode_len_dev")

    def offsets_dev(self, enc_len, out_off, cap_off=None, base: int = 0, dev: int = 0, stream=None) -> None:
        n = out_off.numel() - 1
        check(self._L.mhq_huff_offsets_dev(self._h, dev, enc_len.data_ptr(), n, base, out_off.data_ptr(),
                                           cap_off.data_ptr() if cap_off is not None else None,
                                           self._stream(stream)), "offsets_dev")

    def encode_layout_dev(self, data, off, enc_len, out_off, cap_off=None, base: int = 0, dev: int = 0,
                          stream=None) -> None:
        """encode_len_dev + offsets_dev in two launches (the scan's first pass
        is folded into the sizing kernel)."""
        n = off.numel() - 1
        check(self._L.mhq_huff_encode_layout_dev(self._h, dev, data.data_ptr(), off.data_ptr(), n, base,
                                                 enc_len.data_ptr(), out_off.data_ptr(),
                                                 cap_off.data_ptr() if cap_off is not None else None,
                                                 self._stream(stream)), "encode_layout_dev")

    def bound_call(self, name: str, *args):
        """A zero-argument callable that calls the C entry point `name` with
        `args` converted to their C types once (device pointers and sizes that
        stay the same from call to call), raising MhqError on a failure.  The
        per-call host cost is then about a cgo call's -- what the Go host of
        INTEGRATION.md pays -- not ctypes' argument conversion (bench.py's
        timed steps repeat the same calls on the same buffers)."""
        fn = getattr(self._L, name)
        conv = tuple(a if isinstance(a, C._SimpleCData) else t(a) for t, a in zip(fn.argtypes, args))

        def call():
            rc = fn(*conv)
            if rc:
                raise MhqError(rc, name)

        return call

    def bind_encode_packed_dev(self, data, off, in_bytes: int, enc_len, out_off, cap_off, out, base: int = 0,
                               dev: int = 0, stream=None):
        """encode_packed_dev's call, bound (bound_call) for repeated use."""
        if out.element_size() != 1:
            raise TypeError("encode_packed_dev: out must be a byte tensor")
        return self.bound_call("mhq_huff_encode_packed_dev", self._h, dev, data.data_ptr(), off.data_ptr(),
                               off.numel() - 1, in_bytes, base, enc_len.data_ptr(), out_off.data_ptr(),
                               cap_off.data_ptr() if cap_off is not None else None, out.data_ptr(), out.numel(),
                               self._stream(stream))

    def bind_decode_dev(self, enc, off, out, cap_off, out_len, status, dev: int = 0, stream=None):
        """decode_dev's call, bound (bound_call) for repeated use."""
        return self.bound_call("mhq_huff_decode_dev", self._h, dev, enc.data_ptr(), off.data_ptr(), off.numel() - 1,
                               out.data_ptr(), cap_off.data_ptr(), out_len.data_ptr(), status.data_ptr(),
                               self._stream(stream))

    def encode_packed_dev(self, data, off, in_bytes: int, enc_len, out_off, cap_off, out, base: int = 0,
                          dev: int = 0, stream=None) -> None:
        """encode_layout_dev + encode_dev in one call (one launch for short
        literals); out (uint8) must hold 30 * in_bytes // 8 + n bytes."""
        n = off.numel() - 1
        if out.element_size() != 1:
            raise TypeError("encode_packed_dev: out must be a byte tensor")
        check(self._L.mhq_huff_encode_packed_dev(self._h, dev, data.data_ptr(), off.data_ptr(), n, in_bytes, base,
                                                 enc_len.data_ptr(), out_off.data_ptr(),
                                                 cap_off.data_ptr() if cap_off is not None else None,
                                                 out.data_ptr(), out.numel(), self._stream(stream)),
              "encode_packed_dev")

    def capacity_dev(self, in_off, cap_off, base: int = 0, dev: int = 0, stream=None) -> None:
        n = in_off.numel() - 1
        check(self._L.mhq_huff_capacity_dev(self._h, dev, in_off.data_ptr(), n, base, cap_off.data_ptr(),
                                            self._stream(stream)), "capacity_dev")

    def encode_dev(self, data, off, out, out_off, dev: int = 0, stream=None) -> None:
        n = off.numel() - 1
        check(self._L.mhq_huff_encode_dev(self._h, dev, data.data_ptr(), off.data_ptr(), n, out.data_ptr(),
                                          out_off.data_ptr(), self._stream(stream)), "encode_dev")

    def decode_dev(self, enc, off, out, cap_off, out_len, status, dev: int = 0, stream=None,
                   in_bytes: int = 0) -> None:
        """mhq_huff_decode_dev; with in_bytes (the batch's encoded bytes,
        off[n] - off[0]) mhq_huff_decode_sized_dev, which picks the
        long-literal form for a mean literal over 64 encoded bytes."""
        n = off.numel() - 1
        if in_bytes:
            check(self._L.mhq_huff_decode_sized_dev(self._h, dev, enc.data_ptr(), off.data_ptr(), n, in_bytes,
                                                    out.data_ptr(), cap_off.data_ptr(), out_len.data_ptr(),
                                                    status.data_ptr(), self._stream(stream)), "decode_sized_dev")
            return
        check(self._L.mhq_huff_decode_dev(self._h, dev, enc.data_ptr(), off.data_ptr(), n, out.data_ptr(),
                                          cap_off.data_ptr(), out_len.data_ptr(), status.data_ptr(),
                                          self._stream(stream)), "decode_dev")

    def read_strings_dev(self, blk, pos, limit, prefix, out, out_off, out_len, status, nxt, dev: int = 0,
                         stream=None) -> None:
        n = pos.numel()
        check(self._L.mhq_read_strings_dev(self._h, dev, blk.data_ptr(), blk.numel(), pos.data_ptr(),
                                           limit.data_ptr(), prefix.data_ptr(), n, out.data_ptr(), out.numel(),
                                           out_off.data_ptr(), out_len.data_ptr(), status.data_ptr(),
                                           nxt.data_ptr(), self._stream(stream)), "read_strings_dev")

    def read_ints_dev(self, blk, pos, limit, prefix, value, nxt, status, index: bool = False, dev: int = 0,
                      stream=None) -> None:
        n = pos.numel()
        check(self._L.mhq_read_ints_dev(self._h, dev, blk.data_ptr(), pos.data_ptr(), limit.data_ptr(),
                                        prefix.data_ptr(), n, 1 if index else 0, value.data_ptr(), nxt.data_ptr(),
                                        status.data_ptr(), self._stream(stream)), "read_ints_dev")

    def read_varints_dev(self, blk, pos, limit, value, nxt, status, dev: int = 0, stream=None) -> None:
        n = pos.numel()
        check(self._L.mhq_read_varints_dev(self._h, dev, blk.data_ptr(), pos.data_ptr(), limit.data_ptr(), n,
                                           value.data_ptr(), nxt.data_ptr(), status.data_ptr(),
                                           self._stream(stream)), "read_varints_dev")


_default: Optional[Codec] = None


def default_codec() -> Codec:
    global _default
    if _default is None:
        _default = Codec()
    return _default


def code_table() -> Tuple[List[int], List[int]]:
    """The kernels' code table (hc/huffmantable.go:9-267) as (len[], code[])."""
    L = _lib.load()
    ln = (C.c_uint8 * 256)()
    code = (C.c_uint32 * 256)()
    check(L.mhq_code_table(ln, code), "mhq_code_table")
    return list(ln), list(code)


# ------------------------------------------------------------------------
# The batch entry points the cgo shim adds to package hc.
# ------------------------------------------------------------------------
def HuffmanEncodeBatch(lits: Sequence[bytes], codec: Optional[Codec] = None) -> List[bytes]:
    """Per literal: HuffmanCompressor.Write(l) then Pad() (hc/huffman.go:23-37)."""
    codec = codec or default_codec()
    data, off = pack(lits)
    enc, enc_off = codec.encode(data, off)
    return unpack(enc, enc_off)


def HuffmanDecodeBatch(enc: Sequence[bytes], codec: Optional[Codec] = None
                       ) -> Tuple[List[bytes], List[Optional[Exception]]]:
    """Per literal: HuffmanDecompressor.Read until EOF (hc/huffman.go:102-121)."""
    codec = codec or default_codec()
    data, off = pack(enc)
    out, cap_off, out_len, status = codec.decode(data, off)
    vals = unpack(out, cap_off, out_len)
    errs = [InvalidHuffmanCoding() if s == _lib.MHQ_LIT_INVALID else None for s in status]
    return vals, errs


class StringEOF(EOFError):
    """io.EOF from Reader.ReadString (hc/io.go:92-94)."""


def ReadStringBatch(blk: bytes, pos: Sequence[int], prefix: Sequence[int], limit: Optional[Sequence[int]] = None,
                    codec: Optional[Codec] = None) -> Tuple[List[bytes], List[Optional[Exception]], List[int]]:
    """Per literal: Reader.ReadString(prefix[i]) at pos[i] (hc/io.go:73-97);
    returns (values, errors, next positions)."""
    codec = codec or default_codec()
    vals, status, nxt = codec.read_strings(blk, pos, prefix, limit)
    errs: List[Optional[Exception]] = []
    for st in status:
        errs.append(InvalidHuffmanCoding() if st == _lib.MHQ_STR_INVALID
                    else StringEOF() if st == _lib.MHQ_STR_EOF
                    else RuntimeError("output buffer too small") if st == _lib.MHQ_STR_NOSPACE else None)
    return vals, errs, [int(x) for x in nxt]


def WriteStringRawBatch(strs: Sequence[bytes], prefix: Sequence[int], choice: int = HuffmanCodingAuto,
                        lead: Optional[Sequence[int]] = None, codec: Optional[Codec] = None) -> List[bytes]:
    """Per string: Writer.WriteStringRaw(s, prefix[i], choice) (hc/io.go:153-197),
    the frame starting with opcode bits lead[i] above the H bit."""
    codec = codec or default_codec()
    return codec.write_strings(strs, prefix, lead, choice)


class IntegerOverflow(OverflowError):
    """ErrIntegerOverflow (hc/io.go:12)."""

    def __init__(self):
        super().__init__("integer overflow")


def ReadIntBatch(blk: bytes, pos: Sequence[int], prefix: Sequence[int], limit: Optional[Sequence[int]] = None,
                 index: bool = False, codec: Optional[Codec] = None):
    """Per integer: Reader.ReadInt(prefix[i]) (ReadIndex with index=True) at
    pos[i] (hc/io.go:25-67); returns (values, errors, next positions)."""
    codec = codec or default_codec()
    vals, status, nxt = codec.read_ints(blk, pos, prefix, limit, index)
    errs: List[Optional[Exception]] = []
    for st in status:
        errs.append(IntegerOverflow() if st == _lib.MHQ_INT_OVERFLOW
                    else EOFError("EOF") if st == _lib.MHQ_INT_EOF
                    else ValueError("prefix outside 1..8") if st == _lib.MHQ_INT_BADARG else None)
    return vals, errs, nxt


def WriteIntBatch(values: Sequence[int], prefix: Sequence[int], lead: Optional[Sequence[int]] = None,
                  codec: Optional[Codec] = None) -> List[bytes]:
    """Per integer: Writer.WriteInt(v, prefix[i]) after opcode bits lead[i] (hc/io.go:110-137)."""
    codec = codec or default_codec()
    return codec.write_ints(values, prefix, lead)


def HuffmanChoose(raw_len: int, enc_len: int, choice: int = HuffmanCodingAuto) -> bool:
    """Whether WriteStringRaw sends the Huffman form (hc/io.go:156-178)."""
    if choice == HuffmanCodingNever:
        return False
    return choice == HuffmanCodingAlways or enc_len < raw_len
