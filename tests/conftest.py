import os
import sys

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if REPO not in sys.path:
    sys.path.insert(0, REPO)

GOLDEN = os.path.join(REPO, "tests", "golden")


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs a gfx950 (MI355X) GPU; parity tests through the C ABI")


@pytest.fixture(scope="session")
def golden():
    import json

    def load(name):
        with open(os.path.join(GOLDEN, name)) as f:
            return json.load(f)

    return load


@pytest.fixture(scope="session")
def oracle_mod():
    from oracle import oracle

    oracle.build()
    return oracle


@pytest.fixture(autouse=True)
def _dbg_bounds_records():
    """With MHQ_DBG_BOUNDS_CHECK=1 and a -DMHQ_DBG_BOUNDS build of the library
    (MHQ_LIB_PATH), every test ends by reading the kernels' bounds records
    (huff_decode_dev.h: LDS records, the fast loop's output word, the decode
    and read path's global stores): none may have been recorded."""
    yield
    crumbs = os.environ.get("MHQ_CRUMBS_OUT")
    if crumbs:  # a -DMHQ_DBG_CRUMBS build: the read path's last global accesses (kept after a GPU fault)
        from minhq_amd import _lib

        fn = getattr(_lib.load(), "mhq_dbg_crumbs_dump", None)
        if fn is not None:
            fn(crumbs.encode())
    if os.environ.get("MHQ_DBG_BOUNDS_CHECK") != "1":
        return
    import ctypes

    from minhq_amd import _lib

    L = _lib.load()
    for name in ("mhq_dbg_bounds_decode", "mhq_dbg_bounds_read"):
        fn = getattr(L, name)
        buf = (ctypes.c_ulonglong * 49)()
        assert fn(buf, 49) == 0, name
        recs = [(int(buf[1 + 3 * k]), hex(buf[2 + 3 * k]), hex(buf[3 + 3 * k])) for k in range(min(16, int(buf[0])))]
        assert int(buf[0]) == 0, f"{name}: {int(buf[0])} bounds violations, first {recs}"
