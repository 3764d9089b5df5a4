"""ctypes binding of libmhq_huff.so -- the same C ABI a cgo shim binds.

Every symbol declared in include/mhq_huff.h is bound here with its exact
signature.  There is no fallback: if the library is missing the import of
any codec entry point raises.
"""
from __future__ import annotations

import ctypes as C
import os

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("MHQ_LIB_PATH") or os.path.join(HERE, "libmhq_huff.so")

MHQ_OK = 0
MHQ_EINVAL = -22
MHQ_ENOMEM = -12
MHQ_ENODEV = -19
MHQ_EHIP = -1000
MHQ_LIT_OK = 0
MHQ_LIT_INVALID = 1
MHQ_STR_OK = 0
MHQ_STR_INVALID = 1
MHQ_STR_EOF = 2
MHQ_STR_NOSPACE = 3
MHQ_INT_OK = 0
MHQ_INT_EOF = 1
MHQ_INT_OVERFLOW = 2
MHQ_INT_BADARG = 3
MHQ_INT_NOSPACE = 4
MHQ_VARINT_OK = 0
MHQ_VARINT_EOF = 1
MHQ_VARINT_TOO_LARGE = 2
MHQ_VARINT_NOSPACE = 3
MHQ_DECODE_AUTO = 0
MHQ_DECODE_TILE = 1
MHQ_DECODE_STREAM = 2

u8p = C.POINTER(C.c_uint8)
u32p = C.POINTER(C.c_uint32)
u64p = C.POINTER(C.c_uint64)
vp = C.c_void_p

# name -> (restype, argtypes); mirrors include/mhq_huff.h one to one.
SIGNATURES = {
    "mhq_open": (C.c_int, [C.POINTER(vp), C.c_int]),
    "mhq_open_devices": (C.c_int, [C.POINTER(vp), C.POINTER(C.c_int), C.c_int]),
    "mhq_close": (None, [vp]),
    "mhq_device_count": (C.c_int, [vp]),
    "mhq_strerror": (C.c_char_p, [C.c_int]),
    "mhq_code_table": (C.c_int, [u8p, u32p]),
    "mhq_host_alloc": (vp, [C.c_size_t]),
    "mhq_host_free": (None, [vp]),
    "mhq_huff_encode_len": (C.c_int, [vp, u8p, u64p, C.c_uint64, u32p]),
    "mhq_huff_encode": (C.c_int, [vp, u8p, u64p, C.c_uint64, u8p, u64p]),
    "mhq_huff_decode": (C.c_int, [vp, u8p, u64p, C.c_uint64, u8p, u64p, u32p, u8p]),
    "mhq_huff_encode_len_dev": (C.c_int, [vp, C.c_int, vp, vp, C.c_uint64, vp, vp]),
    "mhq_huff_offsets_dev": (C.c_int, [vp, C.c_int, vp, C.c_uint64, C.c_uint64, vp, vp, vp]),
    "mhq_huff_encode_layout_dev": (C.c_int, [vp, C.c_int, vp, vp, C.c_uint64, C.c_uint64, vp, vp, vp, vp]),
    "mhq_huff_encode_packed_dev": (C.c_int, [vp, C.c_int, vp, vp, C.c_uint64, C.c_uint64, C.c_uint64, vp, vp, vp,
                                             vp, C.c_uint64, vp]),
    "mhq_huff_capacity_dev": (C.c_int, [vp, C.c_int, vp, C.c_uint64, C.c_uint64, vp, vp]),
    "mhq_huff_encode_dev": (C.c_int, [vp, C.c_int, vp, vp, C.c_uint64, vp, vp, vp]),
    "mhq_huff_decode_dev": (C.c_int, [vp, C.c_int, vp, vp, C.c_uint64, vp, vp, vp, vp, vp]),
    "mhq_huff_decode_sized_dev": (C.c_int, [vp, C.c_int, vp, vp, C.c_uint64, C.c_uint64, vp, vp, vp, vp, vp]),
    "mhq_set_decode_form": (C.c_int, [C.c_int]),
    "mhq_debug_poison_scratch": (C.c_int, [C.c_int]),
    "mhq_read_strings_dev": (C.c_int, [vp, C.c_int, vp, C.c_uint64, vp, vp, vp, C.c_uint64, vp, C.c_uint64,
                                       vp, vp, vp, vp, vp]),
    "mhq_write_strings_dev": (C.c_int, [vp, C.c_int, vp, vp, C.c_uint64, vp, vp, C.c_int, vp, C.c_uint64,
                                        vp, vp, vp]),
    "mhq_read_strings": (C.c_int, [vp, u8p, C.c_uint64, u64p, u64p, u8p, C.c_uint64, u8p, C.c_uint64, u64p,
                                   u32p, u8p, u64p]),
    "mhq_write_strings": (C.c_int, [vp, u8p, u64p, C.c_uint64, u8p, u8p, C.c_int, u8p, C.c_uint64, u64p,
                                    u8p]),
    "mhq_read_ints_dev": (C.c_int, [vp, C.c_int, vp, vp, vp, vp, C.c_uint64, C.c_int, vp, vp, vp, vp]),
    "mhq_write_ints_dev": (C.c_int, [vp, C.c_int, vp, vp, vp, C.c_uint64, vp, C.c_uint64, vp, vp, vp]),
    "mhq_read_ints": (C.c_int, [vp, u8p, C.c_uint64, u64p, u64p, u8p, C.c_uint64, C.c_int, u64p, u64p, u8p]),
    "mhq_write_ints": (C.c_int, [vp, u64p, u8p, u8p, C.c_uint64, u8p, C.c_uint64, u64p, u8p]),
    "mhq_read_varints_dev": (C.c_int, [vp, C.c_int, vp, vp, vp, C.c_uint64, vp, vp, vp, vp]),
    "mhq_read_frames_dev": (C.c_int, [vp, C.c_int, vp, vp, vp, C.c_uint64, vp, vp, vp, vp, vp]),
    "mhq_write_varints_dev": (C.c_int, [vp, C.c_int, vp, C.c_uint64, vp, C.c_uint64, vp, vp, vp]),
    "mhq_read_varints": (C.c_int, [vp, u8p, C.c_uint64, u64p, u64p, C.c_uint64, u64p, u64p, u8p]),
    "mhq_read_frames": (C.c_int, [vp, u8p, C.c_uint64, u64p, u64p, C.c_uint64, u8p, u64p, u64p, u8p]),
    "mhq_write_varints": (C.c_int, [vp, u64p, C.c_uint64, u8p, C.c_uint64, u64p, u8p]),
}

_lib = None


class MhqError(RuntimeError):
    def __init__(self, rc: int, what: str):
        self.rc = rc
        msg = _strerror(rc)
        super().__init__(f"{what}: {msg} (rc={rc})")


def _strerror(rc: int) -> str:
    try:
        return load().mhq_strerror(rc).decode()
    except Exception:  # pragma: no cover
        return "unknown"


def load():
    """Loads the in-tree libmhq_huff.so (raises OSError if it is absent)."""
    global _lib
    if _lib is None:
        # One HIP runtime per process: PyTorch wheels bundle their own
        # libamdhip64 (SONAME libamdhip64.so.7).  Importing torch first makes
        # the dynamic linker bind this library to that same runtime, so torch
        # streams, events and allocations are valid handles here.  Loaded the
        # other way round, torch would bring up a second runtime that finds no
        # GPU.  Without torch (a Go/cgo host) /opt/rocm's runtime is used.
        try:
            import torch  # noqa: F401
        except ImportError:
            pass
        if not os.path.exists(LIB_PATH):
            raise OSError(f"{LIB_PATH} is missing: run `python -m minhq_amd.build` "
                          "(or __graft_entry__.build()) first")
        L = C.CDLL(LIB_PATH)
        for name, (res, args) in SIGNATURES.items():
            fn = getattr(L, name)
            fn.restype = res
            fn.argtypes = args
        _lib = L
    return _lib


def check(rc: int, what: str) -> None:
    if rc != MHQ_OK:
        raise MhqError(rc, what)
