"""ctypes wrapper for oracle/liboracle.so -- TEST INFRASTRUCTURE ONLY.

The CPU restatement of minhq's Go Huffman path (see huff_oracle.c).  Only
tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg import this
module; the product package minhq_amd/ never does.
"""
from __future__ import annotations

import ctypes as C
import os
import subprocess

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
_SO = os.path.join(_HERE, "liboracle.so")

OK = 0
INVALID = 1
ERR_EOF = -1
ERR_TOO_LARGE = -2
ERR_SHORT_WRITE = -3
ERR_OVERFLOW = -4

_lib = None


def build(force: bool = False) -> str:
    """Compile liboracle.so with gcc (oracle/Makefile)."""
    if force or not os.path.exists(_SO):
        subprocess.check_call(["make", "-s", "-C", _HERE, "liboracle.so"])
    return _SO


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(_SO):
            build()
        L = C.CDLL(_SO)
        u8p, u64p, u32p = C.POINTER(C.c_uint8), C.POINTER(C.c_uint64), C.POINTER(C.c_uint32)
        sz, szp = C.c_size_t, C.POINTER(C.c_size_t)
        L.orc_table.argtypes = [u8p, u32p]
        L.orc_tree_nodes.restype = C.c_int
        L.orc_bw_new.restype = C.c_void_p
        L.orc_bw_new.argtypes = [u8p, sz]
        L.orc_bw_write_bits.argtypes = [C.c_void_p, C.c_uint64, C.c_uint8]
        L.orc_bw_pad.argtypes = [C.c_void_p, C.c_uint8]
        L.orc_bw_written.argtypes = [C.c_void_p]
        L.orc_bw_written.restype = sz
        L.orc_bw_free.argtypes = [C.c_void_p]
        L.orc_huff_encoded_len.argtypes = [u8p, sz]
        L.orc_huff_encoded_len.restype = sz
        L.orc_huff_encode.argtypes = [u8p, sz, u8p, sz, szp]
        L.orc_huff_decode.argtypes = [u8p, sz, u8p, sz, szp]
        L.orc_read_string.argtypes = [u8p, sz, C.c_uint8, C.c_uint8, u8p, sz, szp, szp]
        L.orc_write_string.argtypes = [u8p, sz, C.c_uint8, C.c_uint8, C.c_uint8, C.c_int, u8p, sz, szp]
        L.orc_read_int.argtypes = [u8p, sz, C.c_uint8, C.c_uint8, C.POINTER(C.c_uint64), szp]
        L.orc_read_varint.argtypes = [u8p, sz, C.POINTER(C.c_uint64), szp]
        L.orc_write_varint.argtypes = [C.c_uint64, u8p, sz, szp]
        L.orc_read_frame.argtypes = [u8p, sz, C.POINTER(C.c_uint8), C.POINTER(C.c_uint64), szp]
        L.orc_write_int.argtypes = [C.c_uint64, C.c_uint8, C.c_uint8, C.c_uint8, u8p, sz, szp]
        L.orc_encode_len_batch.argtypes = [u8p, u64p, C.c_uint64, u32p, C.c_int]
        L.orc_encode_batch.argtypes = [u8p, u64p, C.c_uint64, u8p, u64p, C.c_int]
        L.orc_decode_batch.argtypes = [u8p, u64p, C.c_uint64, u8p, u64p, u32p, u8p, C.c_int]
        L.orc_decode_fast_batch.argtypes = [u8p, u64p, C.c_uint64, u8p, u64p, u32p, u8p, C.c_int]
        L.orc_huff_decode_fast.argtypes = [u8p, sz, u8p, sz, szp]
        _lib = L
    return _lib


def _buf(b: bytes):
    n = len(b)
    arr = (C.c_uint8 * max(n, 1)).from_buffer_copy(b if n else b"\0")
    return arr


def _ptr(a: np.ndarray, ctype):
    return a.ctypes.data_as(C.POINTER(ctype))


def table():
    L = lib()
    ln = (C.c_uint8 * 256)()
    val = (C.c_uint32 * 256)()
    L.orc_table(ln, val)
    return list(ln), list(val)


def tree_nodes() -> int:
    return lib().orc_tree_nodes()


def encoded_len(s: bytes) -> int:
    return lib().orc_huff_encoded_len(_buf(s), len(s))


def encode(s: bytes) -> bytes:
    """HuffmanCompressor.Write + Pad (hc/huffman.go:23-37)."""
    L = lib()
    cap = L.orc_huff_encoded_len(_buf(s), len(s))
    out = (C.c_uint8 * max(cap, 1))()
    got = C.c_size_t(0)
    rc = L.orc_huff_encode(_buf(s), len(s), out, cap, C.byref(got))
    if rc:
        raise RuntimeError(f"oracle encode rc={rc}")
    return bytes(out[: got.value])


def decode(enc: bytes, cap: int | None = None):
    """HuffmanDecompressor.Read to EOF (hc/huffman.go:102-121).

    Returns (bytes, status) with status OK or INVALID; the bytes are those
    produced before the error, as Read returns them.
    """
    L = lib()
    if cap is None:
        cap = len(enc) * 8 // 5 + 1  # hc/io.go:87
    out = (C.c_uint8 * max(cap, 1))()
    got = C.c_size_t(0)
    st = L.orc_huff_decode(_buf(enc), len(enc), out, cap, C.byref(got))
    return bytes(out[: got.value]), st


def read_int(data: bytes, prefix: int, skip_bits: int = 0):
    """Reader.ReadInt (hc/io.go:25-55) after skip_bits opcode bits:
    returns (value, rc, consumed octets); rc 0 OK, ERR_EOF or ERR_OVERFLOW."""
    L = lib()
    v, used = C.c_uint64(0), C.c_size_t(0)
    rc = L.orc_read_int(_buf(data), len(data), skip_bits, prefix, C.byref(v), C.byref(used))
    return v.value, rc, used.value


def write_int(v: int, prefix: int, lead: int = 0, lead_bits: int = 0) -> bytes:
    """Writer.WriteInt (hc/io.go:110-137) after lead_bits opcode bits."""
    L = lib()
    out = (C.c_uint8 * 16)()
    got = C.c_size_t(0)
    rc = L.orc_write_int(C.c_uint64(v), lead, lead_bits, prefix, out, 16, C.byref(got))
    if rc:
        raise RuntimeError(f"oracle write_int rc={rc}")
    return bytes(out[: got.value])


def read_varint(data: bytes):
    """ReadVarint (frame.go:72-79): (value, rc, consumed)."""
    L = lib()
    v, used = C.c_uint64(0), C.c_size_t(0)
    rc = L.orc_read_varint(_buf(data), len(data), C.byref(v), C.byref(used))
    return v.value, rc, used.value


def write_varint(v: int):
    """WriteVarint (frame.go:128-152): (bytes, rc); rc ERR_TOO_LARGE for v >= 2^62."""
    L = lib()
    out = (C.c_uint8 * 8)()
    got = C.c_size_t(0)
    rc = L.orc_write_varint(C.c_uint64(v), out, 8, C.byref(got))
    return bytes(out[: got.value]), rc


def read_frame(data: bytes):
    """ReadFrame's header (frame.go:81-92): (type, payload length, header length, rc)."""
    L = lib()
    t, pl, hl = C.c_uint8(0), C.c_uint64(0), C.c_size_t(0)
    rc = L.orc_read_frame(_buf(data), len(data), C.byref(t), C.byref(pl), C.byref(hl))
    return t.value, pl.value, hl.value, rc


def read_string(data: bytes, prefix: int = 7, skip_bits: int = 0):
    """Reader.ReadString (hc/io.go:73-97): returns (value, rc, consumed)."""
    L = lib()
    cap = max(len(data) * 8 // 5 + 2, 1)
    out = (C.c_uint8 * cap)()
    got, used = C.c_size_t(0), C.c_size_t(0)
    rc = L.orc_read_string(_buf(data), len(data), skip_bits, prefix, out, cap, C.byref(got), C.byref(used))
    return bytes(out[: got.value]), rc, used.value


def write_string(s: bytes, prefix: int = 7, choice: int = 0, lead: int = 0, lead_bits: int = 0) -> bytes:
    """Writer.WriteStringRaw (hc/io.go:153-197); choice 0 Auto 1 Always 2 Never."""
    L = lib()
    cap = len(s) * 4 + 16
    out = (C.c_uint8 * cap)()
    got = C.c_size_t(0)
    rc = L.orc_write_string(_buf(s), len(s), lead, lead_bits, prefix, choice, out, cap, C.byref(got))
    if rc:
        raise RuntimeError(f"oracle write_string rc={rc}")
    return bytes(out[: got.value])


class BitWriter:
    """bitWriter over a fixed buffer (io/bitio.go:17-149)."""

    def __init__(self, cap: int = 256):
        self._out = (C.c_uint8 * cap)()
        self._w = lib().orc_bw_new(self._out, cap)

    def write_bits(self, v: int, count: int) -> int:
        return lib().orc_bw_write_bits(self._w, v, count)

    def write_bit(self, b: int) -> int:
        return self.write_bits(b, 1)

    def pad(self, p: int) -> int:
        return lib().orc_bw_pad(self._w, p)

    def bytes(self) -> bytes:
        return bytes(self._out[: lib().orc_bw_written(self._w)])

    def __del__(self):
        try:
            lib().orc_bw_free(self._w)
        except Exception:
            pass


# ---- batch drivers (numpy arrays; offsets are uint64 of length n+1) ----

def encode_len_batch(data: np.ndarray, off: np.ndarray, nthreads: int = 1) -> np.ndarray:
    n = len(off) - 1
    out = np.zeros(n, dtype=np.uint32)
    lib().orc_encode_len_batch(_ptr(data, C.c_uint8), _ptr(off, C.c_uint64), n, _ptr(out, C.c_uint32), nthreads)
    return out


def encode_batch(data: np.ndarray, off: np.ndarray, out_off: np.ndarray, nthreads: int = 1) -> np.ndarray:
    n = len(off) - 1
    out = np.zeros(max(int(out_off[-1]), 1), dtype=np.uint8)
    rc = lib().orc_encode_batch(_ptr(data, C.c_uint8), _ptr(off, C.c_uint64), n, _ptr(out, C.c_uint8),
                                _ptr(out_off, C.c_uint64), nthreads)
    if rc:
        raise RuntimeError(f"oracle encode_batch rc={rc}")
    return out[: int(out_off[-1])]


def decode_batch(enc: np.ndarray, off: np.ndarray, cap_off: np.ndarray, nthreads: int = 1, fast: bool = False):
    """Restated Go decode per literal (fast=True: the table-driven decoder,
    same results; a CPU baseline, not a checker)."""
    n = len(off) - 1
    out = np.zeros(max(int(cap_off[-1]), 1), dtype=np.uint8)
    out_len = np.zeros(n, dtype=np.uint32)
    status = np.zeros(n, dtype=np.uint8)
    (lib().orc_decode_fast_batch if fast else lib().orc_decode_batch)(_ptr(enc, C.c_uint8), _ptr(off, C.c_uint64), n, _ptr(out, C.c_uint8),
                           _ptr(cap_off, C.c_uint64), _ptr(out_len, C.c_uint32), _ptr(status, C.c_uint8),
                           nthreads)
    return out, out_len, status
