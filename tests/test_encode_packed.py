"""mhq_huff_encode_packed_dev: the encode side of a batch in one call (one
launch for short literals, enc_packed.hip) against the oracle -- enc_len,
out_off, cap_off and every encoded byte -- on the shapes that reach each of
its paths: staged ranges, ranges too long to stage (a long literal among short
ones), output too long for the staging slice, empty literals, partial last
ranges, grids far larger than one resident generation (look-back windows
over many predecessors), a base offset, no cap_off, and batches of longer
literals (the layout + encode path).  Reference: hc/huffman.go:23-37,
hc/io.go:157-172."""
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


def _run(codec, oracle_mod, data, off, base=0, with_cap=True, stream=None):
    import torch

    dev = torch.device("cuda:0")
    n = len(off) - 1
    in_bytes = int(off[-1] - off[0])
    t_data = torch.from_numpy(np.ascontiguousarray(data, dtype=np.uint8).copy()).to(dev)
    if t_data.numel() == 0:
        t_data = torch.zeros(1, dtype=torch.uint8, device=dev)
    t_off = torch.from_numpy(off.astype(np.uint64).view(np.int64).copy()).to(dev)
    enc_len = torch.full((max(n, 1),), -1, dtype=torch.int32, device=dev)
    out_off = torch.full((n + 1,), -1, dtype=torch.int64, device=dev)
    cap_off = torch.full((n + 1,), -1, dtype=torch.int64, device=dev) if with_cap else None
    cap = 30 * in_bytes // 8 + n  # the most n literals of in_bytes bytes encode to (include/mhq_huff.h)
    out = torch.full((max(cap, 1),), 0xA5, dtype=torch.uint8, device=dev)
    torch.cuda.synchronize()  # (the inputs' copies are on the current stream)
    codec.encode_packed_dev(t_data, t_off, in_bytes, enc_len, out_off, cap_off, out, base=base, stream=stream)
    torch.cuda.synchronize()
    ref_len = oracle_mod.encode_len_batch(data, off, nthreads=8) if n else np.zeros(0, np.uint32)
    eoff = np.zeros(n + 1, dtype=np.uint64)
    eoff[1:] = np.cumsum(ref_len, dtype=np.uint64)
    coff = np.zeros(n + 1, dtype=np.uint64)
    coff[1:] = np.cumsum(ref_len.astype(np.uint64) * 8 // 5, dtype=np.uint64)
    ref_enc = oracle_mod.encode_batch(data, off, eoff, nthreads=8) if n else np.zeros(0, np.uint8)
    assert np.array_equal(enc_len.cpu().numpy()[:n].view(np.uint32), ref_len)
    assert np.array_equal(out_off.cpu().numpy().view(np.uint64), eoff + base)
    if with_cap:
        assert np.array_equal(cap_off.cpu().numpy().view(np.uint64), coff + base)
    got = out.cpu().numpy()
    assert got[: int(eoff[-1])].tobytes() == ref_enc.tobytes()


@pytest.mark.parametrize("shape", ["northstar", "config2", "print", "qif_short", "odd_n", "mean37", "mean40"])
def test_packed_short_shapes(codec, oracle_mod, shape):
    """mean37: the four-workgroup shape's largest mean for 512-literal ranges
    (19-20 KB in its 20,224-B staging); mean40: its 448-literal ranges."""
    from minhq_amd import workloads as w

    if shape == "northstar":
        b = w.north_star(1 << 17)
    elif shape == "config2":
        b = w.config2(1 << 17)
    elif shape == "print":
        b = w.config2(1 << 16, "print")
    elif shape == "qif_short":
        b = w.make_batch(50000, "uniform", "hdr", 41, 0, 26)
    elif shape == "mean37":
        b = w.make_batch(1 << 16, "uniform", "hdr", 43, 30, 44)
    elif shape == "mean40":
        b = w.make_batch(1 << 16, "uniform", "hdr", 44, 24, 56)
    else:
        b = w.make_batch(512 * 37 + 311, "uniform", "hdr", 42, 0, 70)
    mean = int(b.off[-1] - b.off[0]) / max(b.n, 1)
    if shape == "mean37":
        assert 36.0 <= mean <= 37.5, mean
    if shape == "mean40":
        assert 37.5 < mean <= 40.0, mean
    _run(codec, oracle_mod, b.data, b.off)


def test_packed_many_ranges_base_no_cap(codec, oracle_mod):
    """2^20 literals: 2048 ranges, far more than one resident generation, so
    look-backs cross windows of 512 predecessors; a base offset; no cap_off."""
    from minhq_amd import workloads as w

    b = w.north_star(1 << 20)
    _run(codec, oracle_mod, b.data, b.off, base=12345, with_cap=False)


def test_packed_unstaged_ranges(codec, oracle_mod):
    """Ranges whose plaintext exceeds the 24 KiB staging slice (a 3 KB
    literal every 700, a 40 KB one once) or whose output exceeds the 20 KiB
    output slice (random bytes: 30-bit codes), sized and encoded per literal
    from global memory; empty literals throughout."""
    from minhq_amd import hc, workloads as w

    rng = np.random.default_rng(43)
    b = w.make_batch(30000, "uniform", "hdr", 43, 0, 40)
    lits = hc.unpack(b.data, b.off)
    for i in range(0, len(lits), 700):
        lits[i] = bytes(rng.integers(32, 127, 3000, dtype=np.uint8))
    lits[12000] = bytes(rng.integers(0, 256, 40000, dtype=np.uint8))
    for i in range(25000, 25512):  # one range of random bytes: ~3.7x expansion, its output over the slice
        lits[i] = bytes(rng.integers(0, 256, 40, dtype=np.uint8))
    for i in range(5, len(lits), 97):
        lits[i] = b""
    data, off = hc.pack(lits)
    _run(codec, oracle_mod, data, off)


@pytest.mark.parametrize("shape", ["r512", "r448"])
def test_packed_overflow_ranges_in_halves(codec, oracle_mod, shape):
    """Ranges over the 20,224-B plaintext staging in batches whose mean keeps
    the four-workgroup shape (512- and 448-literal ranges): each is sized and
    encoded in two staged halves.  Both halves fit (blocks of 30-60-B
    literals); only the second fits (a 15-KB literal in the first); the
    plaintext fits but the codes overflow the 15,360-B output staging (random
    bytes: 30-bit codes); empty literals throughout."""
    from minhq_amd import hc, workloads as w

    R = 512 if shape == "r512" else 448
    rng = np.random.default_rng(49)
    n = 24 * R
    b = w.make_batch(n, "clustered", "hdr", 49, 30, 60) if shape == "r512" else \
        w.make_batch(n, "uniform", "hdr", 49, 30, 46)
    lits = hc.unpack(b.data, b.off)
    for i in range(5 * R, 6 * R):  # both halves fit
        lits[i] = bytes(rng.integers(97, 123, 58, dtype=np.uint8))
    lits[9 * R + 3] = bytes(rng.integers(32, 127, 15000, dtype=np.uint8))  # the first half overflows
    for i in range(13 * R, 14 * R):  # codes over the output staging
        lits[i] = bytes(rng.integers(0, 256, 41, dtype=np.uint8))
    for i in range(7, n, 89):
        lits[i] = b""
    data, off = hc.pack(lits)
    mean = (off[-1] - off[0]) / n
    assert (mean <= 37.5) == (shape == "r512") and mean <= 40, mean  # the shape under test
    _run(codec, oracle_mod, data, off)


def test_packed_staged_long_codes(codec, oracle_mod):
    """Short literals with a sprinkling of bytes whose codes exceed 24 bits
    (control and high bytes: the packed LDS table holds only the length for
    them, the code comes from the global table) in staged ranges."""
    from minhq_amd import hc, workloads as w

    rng = np.random.default_rng(45)
    b = w.north_star(60000)
    lits = hc.unpack(b.data, b.off)
    for i in range(0, len(lits), 3):
        x = bytearray(lits[i])
        for _ in range(max(1, len(x) // 12)):
            x[int(rng.integers(0, len(x)))] = int(rng.choice([0, 1, 9, 10, 13, 22, 127, 128, 200, 254, 255]))
        lits[i] = bytes(x)
    data, off = hc.pack(lits)
    _run(codec, oracle_mod, data, off)


def test_packed_long_literals_path(codec, oracle_mod):
    """Mean literal over 40 bytes: the layout call and the encode, same results."""
    from minhq_amd import workloads as w

    b = w.make_batch(20000, "uniform", "hdr", 44, 30, 200)
    _run(codec, oracle_mod, b.data, b.off, base=7)


def test_packed_tiny_batches(codec, oracle_mod):
    from minhq_amd import hc

    _run(codec, oracle_mod, np.zeros(0, np.uint8), np.zeros(1, np.uint64), base=3)
    for lits in ([b""], [b"a"], [b"", b"", b""], [bytes(range(256))], [b"www.example.com"] * 513):
        data, off = hc.pack(lits)
        _run(codec, oracle_mod, data, off)


@pytest.mark.parametrize("n", [1, 447, 448, 449, 895, 896, 3 * 448 + 17, 100003])
def test_packed_short_ranges_edges(codec, oracle_mod, n):
    """Means of 38-40 B take 448-literal ranges: batches at and around its
    multiples, partial last ranges, one literal."""
    from minhq_amd import workloads as w

    b = w.make_batch(n, "uniform", "hdr", 45 + n % 7, 34, 44)
    mean = int(b.off[-1] - b.off[0]) / max(b.n, 1)
    if n >= 447:
        assert 37.5 < mean <= 40.0, mean
    _run(codec, oracle_mod, b.data, b.off, base=7)


def test_packed_repeated_calls_two_streams(codec, oracle_mod):
    """Calls back to back on one stream (the stream's look-back slots hold the
    previous call's tags) and alternating over two streams."""
    import torch

    from minhq_amd import workloads as w

    s2 = torch.cuda.Stream()
    for k in range(4):
        b = w.north_star(100000 + 1000 * k)
        _run(codec, oracle_mod, b.data, b.off, stream=None if k % 2 == 0 else s2.cuda_stream)


def test_packed_concurrent_launches_four_streams(codec, oracle_mod):
    """Twelve 2^18-literal encodes in flight at once over four streams, no
    synchronisation between them: concurrent launches share the CUs, and a
    range is claimed by ticket (enc_packed.hip), so a workgroup never waits on
    a range no running workgroup holds.  Every call against the oracle."""
    import torch

    from minhq_amd import workloads as w

    dev = torch.device("cuda:0")
    streams = [torch.cuda.Stream().cuda_stream for _ in range(4)]
    b = w.north_star(1 << 18)
    n, in_bytes = b.n, int(b.off[-1])
    t_data = torch.from_numpy(b.data.copy()).to(dev)
    t_off = torch.from_numpy(b.off.view(np.int64).copy()).to(dev)
    cap = 30 * in_bytes // 8 + n
    calls = [(torch.full((n,), -1, dtype=torch.int32, device=dev), torch.full((n + 1,), -1, dtype=torch.int64,
                                                                              device=dev),
              torch.full((cap,), 0xA5, dtype=torch.uint8, device=dev)) for _ in range(12)]
    torch.cuda.synchronize()
    for k, (enc_len, out_off, out) in enumerate(calls):
        codec.encode_packed_dev(t_data, t_off, in_bytes, enc_len, out_off, None, out, base=k,
                                stream=streams[k % 4])
    torch.cuda.synchronize()
    ref_len = oracle_mod.encode_len_batch(b.data, b.off, nthreads=8)
    eoff = np.zeros(n + 1, dtype=np.uint64)
    eoff[1:] = np.cumsum(ref_len, dtype=np.uint64)
    ref_enc = oracle_mod.encode_batch(b.data, b.off, eoff, nthreads=8).tobytes()
    for k, (enc_len, out_off, out) in enumerate(calls):
        assert np.array_equal(enc_len.cpu().numpy().view(np.uint32), ref_len), k
        assert np.array_equal(out_off.cpu().numpy().view(np.uint64), eoff + k), k
        assert out.cpu().numpy()[: int(eoff[-1])].tobytes() == ref_enc, k


def test_packed_rejects_small_out(codec):
    import torch

    from minhq_amd import _lib, workloads as w

    b = w.north_star(1000)
    dev = torch.device("cuda:0")
    t_data = torch.from_numpy(b.data.copy()).to(dev)
    t_off = torch.from_numpy(b.off.view(np.int64).copy()).to(dev)
    in_bytes = int(b.off[-1])
    enc_len = torch.empty(1000, dtype=torch.int32, device=dev)
    out_off = torch.empty(1001, dtype=torch.int64, device=dev)
    out = torch.empty(30 * in_bytes // 8 + 1000 - 1, dtype=torch.uint8, device=dev)
    with pytest.raises(_lib.MhqError):
        codec.encode_packed_dev(t_data, t_off, in_bytes, enc_len, out_off, None, out)


@pytest.mark.parametrize("form", ["packed", "layout"])
def test_packed_worst_case_padding_at_min_cap(codec, oracle_mod, form):
    """Literals made only of bytes 10, 13 and 22 (30-bit codes) pad to whole
    bytes: n literals of L bytes need sum ceil(30 L / 8), up to
    floor(30 in_bytes / 8) + n, more than (30 in_bytes + 7) / 8.
    At exactly the documented minimum out_cap every byte is written, on the
    one-launch path (1-byte literals) and on the layout + encode path (43-byte
    literals: a mean over 40 bytes)."""
    from minhq_amd import hc

    rng = np.random.default_rng(6)
    L = 1 if form == "packed" else 43
    lits = [bytes(rng.choice([10, 13, 22], size=L).astype(np.uint8)) for _ in range(3000)]
    data, off = hc.pack(lits)
    n = len(lits)
    in_bytes = int(off[-1])
    need = sum((30 * len(x) + 7) // 8 for x in lits)
    assert (30 * in_bytes + 7) // 8 < need <= 30 * in_bytes // 8 + n
    _run(codec, oracle_mod, data, off)


def test_packed_in_bytes_mismatch_poisons_out_off(codec):
    """An in_bytes that is not in_off[n] - in_off[0] is caught on the device:
    nothing is encoded and out_off[n] is UINT64_MAX."""
    import torch

    from minhq_amd import workloads as w

    b = w.north_star(5000)
    dev = torch.device("cuda:0")
    t_data = torch.from_numpy(b.data.copy()).to(dev)
    t_off = torch.from_numpy(b.off.view(np.int64).copy()).to(dev)
    in_bytes = int(b.off[-1])
    enc_len = torch.zeros(5000, dtype=torch.int32, device=dev)
    out_off = torch.zeros(5001, dtype=torch.int64, device=dev)
    out = torch.full((30 * in_bytes // 8 + 5000,), 0xA5, dtype=torch.uint8, device=dev)
    codec.encode_packed_dev(t_data, t_off, in_bytes - 100, enc_len, out_off, None, out)
    torch.cuda.synchronize()
    assert int(out_off[-1].item()) == -1  # UINT64_MAX
    assert int((out != 0xA5).sum().item()) == 0


def test_packed_stale_slots_with_next_tag(codec, oracle_mod):
    """Look-back slots left by a larger call can never match a later call's
    tag: the tags are per slot buffer and the buffer is zeroed when it is
    allocated and when its tags wrap (take_slots, mhq_api.cpp).  Poison the
    stream's slot buffer with every tag a later call could use -- here, by
    running many calls of different sizes on one stream, the small ones
    after large ones -- and check each against the oracle."""
    import torch

    from minhq_amd import workloads as w

    s = torch.cuda.Stream().cuda_stream
    for n in (20000, 300, 9000, 77, 20000, 5, 1500):
        b = w.north_star(n)
        _run(codec, oracle_mod, b.data, b.off, stream=s)
