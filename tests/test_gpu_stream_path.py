"""GPU parity of the decode paths that only full-size tile geometry reaches
(VERDICT r01 item 1): `decode_tile_long` with `end_checked_g` and
`OutAccG::finish`, `decode_literal_global`, and `decode_tile_pieces`' single
literal (m == 0) branch, compared with the oracle (restated hc/huffman.go:
102-121) on out_len, status and every decoded byte of a deterministic sample.

The paths are chosen per wave tile (huff_decode.hip decode_kernel): a tile of
`tl` literals whose input overflows 2x the 4 KiB input slice streams through
per-lane windows (decode_tile_long); one within 2x goes in staged pieces, and
a literal larger than a slice alone goes to decode_literal_global (m == 0), as
does any literal whose region is smaller than floor(8C/5) in the long path.
The tests compute the tile geometry the launcher will use and assert it puts
the literals on those paths, so a change of geometry cannot silently turn
them into staged-path tests.

Inputs mix, per the reference rules (hc/huffman.go:104-113):
  valid encodings of random bytes (long codes common);
  0xff-biased garbage (the EOS prefix, with and without a 31st one);
  valid symbols followed by 24..31 one bits (exactly 30 = EOS: INVALID);
  truncating regions (Read stops when the buffer is full);
  regions starting at every byte offset mod 4.
"""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu

KWIN = 4096  # huff_decode.hip kWIn: a wave's input slice (kPF = 4)
KWOUT = 6448  # kWOut
WAVES, TILE = 12, 128  # MHQ_DEC_WAVES, MHQ_DEC_TILE
BIG_LO, BIG_HI = 1900, 2600  # plaintext bytes of the big literals: ~4.1-5.9 KB encoded


@pytest.fixture(scope="module")
def codec():
    from minhq_amd import build, hc

    build.build()
    c = hc.Codec(1)
    yield c
    c.close()


def _tile_len(n, cus, nin, nout):
    """launch_decode's tile length and workgroup range, then decode_kernel's
    own cut for batches whose mean literal overflows the slices."""
    slots = cus * WAVES
    rounds = (n + slots * TILE - 1) // (slots * TILE)
    tl0 = max(1, (n + slots * rounds - 1) // (slots * rounds))
    per_block = (((n + cus - 1) // cus + tl0 - 1) // tl0) * tl0
    ain, aout = (nin + n - 1) // n, (nout + n - 1) // n
    fit = min((KWIN - 16) * 4 // (5 * ain + 8), (KWOUT - 16) * 4 // (5 * aout + 8))
    tl = fit if 64 <= fit < tl0 else tl0
    return tl, per_block


def _tiles(eoff, cap_off, cus):
    n = len(eoff) - 1
    tl, per_block = _tile_len(n, cus, int(eoff[-1] - eoff[0]), int(cap_off[-1] - cap_off[0]))
    starts = []
    for L0 in range(0, n, per_block):
        starts.extend(range(L0, min(L0 + per_block, n), tl))
    s = np.array(starts, dtype=np.int64)
    e = np.minimum(s + tl, (s // per_block) * per_block + per_block)
    return s, np.minimum(e, n)


def _build(rng, oracle_mod, n, plain_lo, plain_hi, kinds, p):
    """A packed batch of n literals: kind 0 valid, 1 garbage, 2 valid + 3 bytes
    of ones, 3 valid with a truncating region.  Returns enc, eoff, cap_off."""
    kind = rng.choice(kinds, size=n, p=p).astype(np.int8)
    L = rng.integers(plain_lo, plain_hi + 1, size=n).astype(np.uint64)
    off = np.zeros(n + 1, dtype=np.uint64)
    off[1:] = np.cumsum(L)
    data = rng.integers(0, 256, size=int(off[-1]), dtype=np.uint8)
    enc_len = oracle_mod.encode_len_batch(data, off, nthreads=8).astype(np.int64)
    eo = np.zeros(n + 1, dtype=np.uint64)
    eo[1:] = np.cumsum(enc_len, dtype=np.uint64)
    enc0 = oracle_mod.encode_batch(data, off, eo, nthreads=8)
    extra = np.where(kind == 2, 3, 0).astype(np.int64)
    C = enc_len + extra
    eoff = np.zeros(n + 1, dtype=np.uint64)
    eoff[1:] = np.cumsum(C, dtype=np.uint64)
    enc = np.full(int(eoff[-1]), 0xFF, dtype=np.uint8)  # appended bytes stay all ones
    # copy the encodings in literal blocks (bounded index arrays)
    B = 1 << 16
    for a in range(0, n, B):
        b = min(a + B, n)
        lo, hi = int(eo[a]), int(eo[b])
        shift = np.repeat((eoff[a:b] - eo[a:b]).astype(np.int64), enc_len[a:b])
        enc[np.arange(lo, hi, dtype=np.int64) + shift] = enc0[lo:hi]
        g = np.repeat(kind[a:b] == 1, C[a:b])  # garbage literals: ones-biased random bytes
        if g.any():
            base = int(eoff[a])
            pos = base + np.flatnonzero(g)
            r = rng.random(pos.size)
            enc[pos] = np.where(r < 0.45, 0xFF, rng.integers(0, 256, pos.size)).astype(np.uint8)
    cap = C * 8 // 5
    cap = np.where(kind == 3, rng.integers(0, np.maximum(cap, 1)), cap)
    gap = rng.integers(0, 4, size=n)  # region starts at every byte offset mod 4
    cap_off = np.zeros(n + 1, dtype=np.uint64)
    cap_off[1:] = np.cumsum(cap + gap, dtype=np.uint64)
    return enc, eoff, cap_off, kind


def _decode_dev(codec, enc, eoff, cap_off):
    import torch

    n = len(eoff) - 1
    dev = torch.device("cuda", 0)
    d_enc = torch.from_numpy(np.concatenate([enc, np.zeros(16, np.uint8)])).to(dev)
    d_eoff = torch.from_numpy(eoff.view(np.int64)).to(dev)
    d_cap = torch.from_numpy(cap_off.view(np.int64)).to(dev)
    out = torch.zeros(int(cap_off[-1]) + 16, dtype=torch.uint8, device=dev)
    out_len = torch.empty(max(n, 1), dtype=torch.int32, device=dev)
    status = torch.empty(max(n, 1), dtype=torch.uint8, device=dev)
    codec.decode_dev(d_enc, d_eoff, out, d_cap, out_len, status)
    torch.cuda.synchronize()
    return out.cpu().numpy(), out_len.cpu().numpy()[:n].astype(np.uint32), status.cpu().numpy()[:n]


def _compare(oracle_mod, enc, eoff, cap_off, out, out_len, status, rng, sample, extra=()):
    out_ref, len_ref, st_ref = oracle_mod.decode_batch(enc, eoff, cap_off, nthreads=8)
    bad = np.flatnonzero((out_len != len_ref) | (status != st_ref))
    assert bad.size == 0, f"{bad.size} literals differ, first {bad[:8]}: " \
        f"len {out_len[bad[:8]]} vs {len_ref[bad[:8]]}, status {status[bad[:8]]} vs {st_ref[bad[:8]]}"
    n = len(eoff) - 1
    idx = np.unique(np.concatenate([rng.choice(n, size=min(sample, n), replace=False), np.arange(min(n, 256)),
                                    np.arange(max(0, n - 256), n), np.asarray(extra, dtype=np.int64)]))
    for i in idx:
        a, m = int(cap_off[i]), int(len_ref[i])
        assert out[a:a + m].tobytes() == out_ref[a:a + m].tobytes(), f"literal {i} bytes differ"
    return st_ref


def test_long_window_path_vs_oracle(codec, oracle_mod):
    """2^20 literals of 128..200 random bytes (~150-350 B encoded): every tile
    is far over 2x the input slice, so each goes through decode_tile_long;
    truncating regions go to decode_literal_global from there."""
    import torch

    rng = np.random.default_rng(20)
    n = 1 << 20
    enc, eoff, cap_off, kind = _build(rng, oracle_mod, n, 128, 200, [0, 1, 2, 3], [0.4, 0.2, 0.2, 0.2])
    cus = torch.cuda.get_device_properties(0).multi_processor_count
    s, e = _tiles(eoff, cap_off, cus)
    tile_in = eoff[e].astype(np.int64) - eoff[s].astype(np.int64)
    long_lits = (e - s)[tile_in > 2 * KWIN].sum()  # only workgroups' last, partial tiles are shorter
    assert long_lits > 0.97 * n, "the tiles would not take the long path"
    out, out_len, status = _decode_dev(codec, enc, eoff, cap_off)
    st = _compare(oracle_mod, enc, eoff, cap_off, out, out_len, status, rng, 6000)
    # the rules really are exercised
    assert (st[kind == 1] != 0).sum() > 1000
    assert (st[kind == 2] != 0).sum() > 1000 and (st[kind == 2] == 0).sum() > 1000
    truncated = (kind == 3) & (out_len < (np.diff(eoff).astype(np.int64) * 8 // 5))
    assert truncated.sum() > 10000


def test_piece_path_single_literal_branch_vs_oracle(codec, oracle_mod):
    """2^20 short literals with a 4.1-5.9 KB literal every ~1500: the tiles
    holding one are over one slice but within two, so they go in staged
    pieces, and the big literal alone overflows a slice (m == 0 ->
    decode_literal_global).  Big ones are valid, garbage or truncated."""
    import torch

    rng = np.random.default_rng(21)
    n = 1 << 20
    enc_s, eoff_s, cap_s, kind_s = _build(rng, oracle_mod, n, 4, 12, [0, 1, 2, 3], [0.85, 0.05, 0.05, 0.05])
    big_at = np.arange(700, n, 1500)
    nb = big_at.size
    enc_b, eoff_b, cap_b, kind_b = _build(rng, oracle_mod, nb, BIG_LO, BIG_HI, [0, 1, 3], [0.4, 0.3, 0.3])
    # splice: literal big_at[k] becomes big literal k (runs of short ones between)
    segs, lens, caps = [], np.diff(eoff_s).astype(np.int64), np.diff(cap_s).astype(np.int64)
    prev = 0
    for k, i in enumerate(big_at):
        segs.append(enc_s[int(eoff_s[prev]):int(eoff_s[i])])
        segs.append(enc_b[int(eoff_b[k]):int(eoff_b[k + 1])])
        lens[i] = int(eoff_b[k + 1] - eoff_b[k])
        caps[i] = int(cap_b[k + 1] - cap_b[k])
        prev = i + 1
    segs.append(enc_s[int(eoff_s[prev]):])
    enc = np.concatenate(segs)
    eoff = np.zeros(n + 1, dtype=np.uint64)
    eoff[1:] = np.cumsum(lens, dtype=np.uint64)
    assert int(eoff[-1]) == enc.size
    cap_off = np.zeros(n + 1, dtype=np.uint64)
    cap_off[1:] = np.cumsum(caps, dtype=np.uint64)
    cus = torch.cuda.get_device_properties(0).multi_processor_count
    s, e = _tiles(eoff, cap_off, cus)
    C = np.diff(eoff).astype(np.int64)
    tile_in = eoff[e].astype(np.int64) - eoff[s].astype(np.int64)
    tile_out = cap_off[e].astype(np.int64) - cap_off[s].astype(np.int64)
    big_tile = np.searchsorted(s, big_at, side="right") - 1
    over = (tile_in[big_tile] + 15 > KWIN) | (tile_out[big_tile] + 15 > KWOUT)
    within = (tile_in[big_tile] <= 2 * KWIN) & (tile_out[big_tile] <= 2 * KWOUT)
    assert (over & within).sum() > nb // 2, "the big literals' tiles would not take the piece path"
    assert (C[big_at] > KWIN - 16).all()  # alone over a slice: m == 0
    out, out_len, status = _decode_dev(codec, enc, eoff, cap_off)
    # every big literal's bytes, and a sample of the rest
    st = _compare(oracle_mod, enc, eoff, cap_off, out, out_len, status, np.random.default_rng(3), 3000, big_at)
    assert (st[big_at] != 0).sum() > 50 and (st[big_at] == 0).sum() > 50


@pytest.mark.parametrize("kind", ["hdr", "adv"])
def test_offsets_past_2gib(codec, oracle_mod, kind):
    """Absolute offsets whose low 32-bit word has bit 31 set (2-4 GiB into the
    buffers): encode writes and decode reads / writes there bit-exactly.  A
    readfirstlane of the low word once sign-extended over the high one, so
    the staged decode path faulted past 2 GiB (config 5's 2.9 GB output)."""
    import torch

    from minhq_amd import workloads

    dev = torch.device("cuda", 0)
    lo, hi = (128, 128) if kind == "adv" else (8, 64)
    b = workloads.make_batch(6000, "fixed" if kind == "adv" else "uniform", kind, 77, lo, hi)
    enc_len = oracle_mod.encode_len_batch(b.data, b.off, nthreads=8)
    eoff = np.zeros(b.n + 1, dtype=np.uint64)
    eoff[1:] = np.cumsum(enc_len, dtype=np.uint64)
    enc_ref = oracle_mod.encode_batch(b.data, b.off, eoff, nthreads=8)
    E = int(eoff[-1])
    cap = np.zeros(b.n + 1, dtype=np.uint64)
    cap[1:] = np.cumsum(np.diff(eoff) * 8 // 5, dtype=np.uint64)
    base_in, base_out = (1 << 31) + 777, 3 * (1 << 30) + 333
    big_in = torch.empty(base_in + E + 16, dtype=torch.uint8, device=dev)
    big_out = torch.empty(base_out + int(cap[-1]) + 16, dtype=torch.uint8, device=dev)
    data = torch.from_numpy(b.data).to(dev)
    off = torch.from_numpy(b.off.view(np.int64)).to(dev)
    # encode into [base_in, base_in + E) of a 2 GiB+ buffer
    eoff_abs = torch.from_numpy((eoff + np.uint64(base_in)).view(np.int64)).to(dev)
    codec.encode_dev(data, off, big_in, eoff_abs)
    torch.cuda.synchronize()
    assert big_in[base_in:base_in + E].cpu().numpy().tobytes() == enc_ref.tobytes()
    # decode from there into [base_out, ...) of a 3 GiB+ buffer
    cap_abs = torch.from_numpy((cap + np.uint64(base_out)).view(np.int64)).to(dev)
    big_out[base_out:base_out + int(cap[-1])].zero_()
    out_len = torch.empty(b.n, dtype=torch.int32, device=dev)
    status = torch.empty(b.n, dtype=torch.uint8, device=dev)
    codec.decode_dev(big_in, eoff_abs, big_out, cap_abs, out_len, status)
    torch.cuda.synchronize()
    assert int(status.sum().item()) == 0
    assert np.array_equal(out_len.cpu().numpy().astype(np.uint64), np.diff(b.off))
    out = big_out[base_out:base_out + int(cap[-1])].cpu().numpy()
    starts = cap[:-1].astype(np.int64)
    lens = np.diff(b.off).astype(np.int64)
    idx = np.repeat(starts - np.cumsum(lens) + lens, lens) + np.arange(int(lens.sum()))
    assert np.array_equal(out[idx], b.data)
