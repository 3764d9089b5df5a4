"""String-literal framing on the GPU: batch Reader.ReadString / Writer.WriteStringRaw
(hc/io.go:73-97, 153-197, with the prefix integers of hc/io.go:25-55, 110-137)
through the C ABI, bit-exact against the CPU oracle (oracle/huff_oracle.c
orc_read_string / orc_write_string) and the reference's own vectors
(hc/io_test.go:77-88, tests/golden/string_vectors.json).
"""
import random

import pytest

pytestmark = pytest.mark.gpu

OK, INVALID, EOF = 0, 1, 2
ORC_EOF, ORC_INVALID = -1, 1


@pytest.fixture(scope="module")
def codec():
    from minhq_amd import build, hc

    build.build()
    c = hc.Codec(1)
    yield c
    c.close()


def _oracle_status(rc):
    return {0: OK, ORC_INVALID: INVALID, ORC_EOF: EOF}[rc]


def test_reference_vectors_read(codec, golden):  # hc/io_test.go:90-101
    vecs = golden("string_vectors.json")
    blk, pos = b"", []
    for v in vecs:  # every literal in a block of its own: limits at its end
        pos.append(len(blk))
        blk += bytes.fromhex(v["hex"])
    limits = pos[1:] + [len(blk)]
    vals, st, nxt = codec.read_strings(blk, pos, [v["prefix"] for v in vecs], limits)
    for v, val, s, e, lim in zip(vecs, vals, st, nxt, limits):
        assert (val, s) == (v["text"].encode(), OK), v["src"]
        assert e == lim


def test_reference_vectors_write(codec, golden):  # hc/io_test.go:103-118: Auto picks the shorter form
    from minhq_amd import hc

    vecs = golden("string_vectors.json")
    raw, huf = {}, {}
    for v in vecs:
        b = bytes.fromhex(v["hex"])
        (huf if b[0] & 0x80 else raw)[v["text"]] = b
    # Auto sends the Huffman form only when it is strictly shorter (hc/io.go:172)
    by_text = {t: huf[t] if len(huf[t]) < len(raw[t]) else raw[t] for t in raw}
    texts = sorted(by_text)
    frames = hc.WriteStringRawBatch([t.encode() for t in texts], [7] * len(texts), codec=codec)
    assert frames == [by_text[t] for t in texts]


def _random_strings(rng, n):
    alpha = b"abcdefghijklmnopqrstuvwxyz0123456789-_./:;=, "
    out = []
    for _ in range(n):
        kind = rng.random()
        L = rng.choice([0, 1, 2, 5, 30, 126, 127, 128, 200, 300]) if kind < 0.3 else rng.randint(0, 60)
        if rng.random() < 0.8:
            out.append(bytes(rng.choice(alpha) for _ in range(L)))
        else:
            out.append(bytes(rng.randrange(256) for _ in range(L)))
    return out


@pytest.mark.parametrize("choice", [0, 1, 2])
def test_write_matches_oracle(codec, oracle_mod, choice):
    rng = random.Random(7 + choice)
    strs = _random_strings(rng, 1500)
    prefixes = [rng.choice([7, 5, 3]) for _ in strs]
    leads = [rng.randrange(1 << (7 - p)) if p < 7 else 0 for p in prefixes]
    frames = codec.write_strings(strs, prefixes, leads, choice)
    for s, p, ld, f in zip(strs, prefixes, leads, frames):
        assert f == oracle_mod.write_string(s, prefix=p, choice=choice, lead=ld, lead_bits=7 - p)


def test_read_matches_oracle(codec, oracle_mod):
    """A block of framed literals (every choice, prefixes 7/5/3, opcode bits
    above): each read from its start to the block end, as the oracle does."""
    rng = random.Random(11)
    strs = _random_strings(rng, 1500)
    blk, pos, prefixes = b"", [], []
    for s in strs:
        p = rng.choice([7, 5, 3])
        ld = rng.randrange(1 << (7 - p)) if p < 7 else 0
        pos.append(len(blk))
        prefixes.append(p)
        blk += oracle_mod.write_string(s, prefix=p, choice=rng.choice([0, 1, 2]), lead=ld, lead_bits=7 - p)
    vals, st, nxt = codec.read_strings(blk, pos, prefixes)
    for i, (s, p) in enumerate(zip(strs, prefixes)):
        ref, rc, used = oracle_mod.read_string(blk[pos[i]:], prefix=p, skip_bits=7 - p)
        assert (vals[i], int(st[i])) == (ref, _oracle_status(rc)), i
        assert vals[i] == s or rc != 0
        assert int(nxt[i]) == pos[i] + used


def test_read_edge_cases(codec, oracle_mod):
    """Truncated blocks, empty literals, invalid codes, header EOF and integer
    overflow -- each checked against the oracle's ReadString restatement."""
    cases = [
        bytes.fromhex("80"),                      # Huffman, length 0: io.EOF
        bytes.fromhex("00"),                      # raw, length 0: ("", nil)
        bytes.fromhex("81ff"),                    # Huffman padding only: io.EOF
        bytes.fromhex("84ffffffff"),              # EOS prefix + a 31st bit: invalid
        bytes.fromhex("843fffffff"),              # "o" then a partial code: ok
        bytes.fromhex("8bc65a283fd29c"),          # Huffman "Hello, World!" cut by the block end
        bytes.fromhex("0d48656c6c"),              # raw cut by the block end
        bytes.fromhex("05"),                      # raw, payload entirely missing: io.EOF
        bytes.fromhex("7f"),                      # length continuation missing: ("", nil)
        bytes.fromhex("7f8080808080808080808002"),  # ReadInt overflow: ("", nil)
        bytes.fromhex("7f00") + b"x" * 127,       # 127-byte raw literal (one continuation octet)
        b"",                                      # nothing to read: ("", nil)
    ]
    for c in cases:
        vals, st, nxt = codec.read_strings(c, [0], [7], [len(c)])
        ref, rc, used = oracle_mod.read_string(c, prefix=7)
        assert (vals[0], int(st[0]), int(nxt[0])) == (ref, _oracle_status(rc), used), c.hex()


def test_read_all_prefixes(codec, oracle_mod):
    rng = random.Random(5)
    for p in range(1, 8):
        strs = _random_strings(rng, 200)
        blk, pos = b"", []
        for s in strs:
            pos.append(len(blk))
            blk += oracle_mod.write_string(s, prefix=p, choice=rng.choice([0, 1, 2]),
                                           lead=rng.randrange(1 << (7 - p)) if p < 7 else 0, lead_bits=7 - p)
        vals, st, _ = codec.read_strings(blk, pos, [p] * len(strs))
        for i, s in enumerate(strs):
            ref, rc, _ = oracle_mod.read_string(blk[pos[i]:], prefix=p, skip_bits=7 - p)
            assert (vals[i], int(st[i])) == (ref, _oracle_status(rc))
            # every literal reads back, except an empty one sent Huffman-coded: io.EOF (hc/io.go:92-94)
            assert vals[i] == s and (int(st[i]) == OK or (s == b"" and int(st[i]) == EOF))


def test_read_limit_past_block_is_einval(codec):
    """mhq_read_strings rejects a limit past the block: the kernels
    would otherwise read beyond the block's device copy."""
    from minhq_amd._lib import MhqError

    blk = bytes.fromhex("8bc65a283fd29c8f65127f1f")
    with pytest.raises(MhqError):
        codec.read_strings(blk, [0], [7], [len(blk) + 1])


def test_read_overlapping_payloads(codec, oracle_mod):
    """Many reads of the same literal (overlapping pos entries): the payloads
    they share add up to more than the block, and each string is still read
    as ReadString would, or reported as NOSPACE -- never cut silently."""
    one = oracle_mod.write_string(b"custom-key: custom-value " * 3, prefix=7, choice=1)
    blk = one + b"\x00" * 4
    n = 64
    vals, st, nxt = codec.read_strings(blk, [0] * n, [7] * n, [len(one)] * n)
    ref, rc, used = oracle_mod.read_string(one, prefix=7)
    assert rc == 0
    NOSPACE = 3
    assert all((v, int(s)) == (ref, OK) or int(s) == NOSPACE for v, s in zip(vals, st))
    assert int(st[0]) == OK and vals[0] == ref


@pytest.mark.parametrize("order", ["in_order", "shuffled", "runs"])
def test_read_gaps_and_order(codec, oracle_mod, order):
    """The decode reads the Huffman payloads where they lie in the block
    (str_frame.hip, launch_decode with in_end): fields separated by other
    octets (gaps), read in block order (tiles staged), in a random order
    (every tile streams), or in shuffled runs of 300 (both kinds of tile).
    Each string against the oracle's ReadString from its position."""
    rng = random.Random({"in_order": 31, "shuffled": 32, "runs": 33}[order])
    strs = _random_strings(rng, 20000)
    blk, pos, prefixes = bytearray(), [], []
    for s in strs:
        blk += bytes(rng.randrange(256) for _ in range(rng.choice([0, 0, 1, 3, 9])))  # a gap
        p = rng.choice([7, 5, 3])
        pos.append(len(blk))
        prefixes.append(p)
        blk += oracle_mod.write_string(s, prefix=p, choice=rng.choice([1, 1, 1, 2, 0]),
                                       lead=rng.randrange(1 << (7 - p)) if p < 7 else 0, lead_bits=7 - p)
    blk = bytes(blk)
    idx = list(range(len(strs)))
    if order == "shuffled":
        rng.shuffle(idx)
    elif order == "runs":
        runs = [idx[k:k + 300] for k in range(0, len(idx), 300)]
        rng.shuffle(runs)
        idx = [i for r in runs for i in r]
    P = [pos[i] for i in idx]
    F = [prefixes[i] for i in idx]
    vals, st, nxt = codec.read_strings(blk, P, F)
    for k, i in enumerate(idx):
        ref, rc, used = oracle_mod.read_string(blk[pos[i]:], prefix=prefixes[i], skip_bits=7 - prefixes[i])
        assert (vals[k], int(st[k])) == (ref, _oracle_status(rc)), (order, k, i)
        assert int(nxt[k]) == pos[i] + used


def test_read_gaps_full_tiles(codec, oracle_mod):
    """Full-size decode tiles over a block with gaps (in order: staged with the
    ends kept apart from the next starts); a sample of strings and every
    status/next against the oracle."""
    import numpy as np

    rng = random.Random(34)
    alpha = b"abcdefghijklmnopqrstuvwxyz0123456789-_./:;=, "
    n = 1 << 18
    blk, pos = bytearray(), []
    pieces = [oracle_mod.write_string(bytes(rng.choice(alpha) for _ in range(rng.randint(1, 40))), prefix=7,
                                      choice=1) for _ in range(4096)]
    for k in range(n):
        if rng.random() < 0.3:
            blk += b"\x82\x90"[: rng.randint(1, 2)]  # other instructions' octets between the fields
        pos.append(len(blk))
        blk += pieces[rng.randrange(len(pieces))] if rng.random() < 0.97 else bytes([0x03]) + b"raw"
    blk = bytes(blk)
    vals, st, nxt = codec.read_strings(blk, pos, [7] * n)
    sample = sorted(rng.sample(range(n), 20000))
    for i in sample:
        ref, rc, used = oracle_mod.read_string(blk[pos[i]:pos[i] + 200], prefix=7)
        assert (vals[i], int(st[i])) == (ref, _oracle_status(rc)), i
        assert int(nxt[i]) == pos[i] + used
    assert (np.asarray(st) == OK).all()


def test_read_full_tiles_long_and_raw(codec, oracle_mod):
    """Full tiles in block order where some tiles hold long strings (too many
    bytes to stage: they stream, their frames parsed from global memory) and
    raw strings in both kinds of tile (payloads copied by the read itself);
    every long or raw string and a sample of the rest against the oracle, every
    status and next."""
    import numpy as np

    rng = random.Random(35)
    alpha = b"abcdefghijklmnopqrstuvwxyz0123456789-_./:;=, "
    n = 1 << 18
    blk, pos, special = bytearray(), [], []
    short = [oracle_mod.write_string(bytes(rng.choice(alpha) for _ in range(rng.randint(0, 40))), prefix=7,
                                     choice=rng.choice([1, 1, 1, 2, 0])) for _ in range(4096)]
    for k in range(n):
        pos.append(len(blk))
        r = rng.random()
        if r < 0.004:  # a long string: its tile streams
            s = bytes(rng.choice(alpha) for _ in range(rng.randint(300, 3000)))
            blk += oracle_mod.write_string(s, prefix=7, choice=rng.choice([1, 2]))
            special.append(k)
        elif r < 0.02:  # raw, maybe binary
            s = bytes(rng.randrange(256) for _ in range(rng.randint(0, 50)))
            blk += oracle_mod.write_string(s, prefix=7, choice=2)
            special.append(k)
        else:
            blk += short[rng.randrange(len(short))]
    blk = bytes(blk)
    vals, st, nxt = codec.read_strings(blk, pos, [7] * n)
    check = sorted(set(special) | set(rng.sample(range(n), 20000)))
    for i in check:
        end = pos[i + 1] if i + 1 < n else len(blk)
        ref, rc, used = oracle_mod.read_string(blk[pos[i]:end], prefix=7)
        assert (vals[i], int(st[i])) == (ref, _oracle_status(rc)), i
        assert int(nxt[i]) == pos[i] + used, i
    assert (np.asarray(nxt, dtype=np.uint64) == np.asarray(pos[1:] + [len(blk)], dtype=np.uint64)).all()
    assert int((np.asarray(st) == EOF).sum()) == sum(1 for i in range(n) if blk[pos[i]] in (0x80,))


def test_read_streamed_then_staged_tiles_every_string(codec, oracle_mod):
    """Regression for the read path's illegal memory access (DESIGN.md, round
    6): a wave's streamed tile (a long string: the frames parsed from global
    memory, lane 0 alone parsing the next tile's first frame, then the
    streamed decode) followed by staged tiles, many times per wave.  Builds
    that called the streamed decode out of line had the register allocator
    copy and spill per-lane values live across the call inside the lane-0
    block, so lanes 1-63 came back with stale registers (the next tile's
    positions and limits, the kinds-shuffle lane of strings 64..127).
    Adjacent strings differ in kind (Huffman OK / empty -> EOF / INVALID,
    raw, raw empty), so a string handled with another lane's state changes its
    (value, status); every string and every next is checked."""
    import numpy as np

    rng = random.Random(61)
    alpha = b"abcdefghijklmnopqrstuvwxyz0123456789-_./:;=, "
    palette = [
        oracle_mod.write_string(b"abc", prefix=7, choice=1),  # Huffman, OK
        bytes([0x80]),  # Huffman, empty: io.EOF
        bytes([0x84, 0xFF, 0xFF, 0xFF, 0xFF]),  # Huffman, the EOS code: INVALID
        bytes([0x03]) + b"xyz",  # raw
        bytes([0x00]),  # raw, empty
        oracle_mod.write_string(b"www.example.com/index.html", prefix=7, choice=1),
    ]
    expect = [oracle_mod.read_string(f, prefix=7) for f in palette]
    n = 1 << 17
    blk, pos, kind, longs = bytearray(), [], [], {}
    for k in range(n):
        pos.append(len(blk))
        if rng.random() < 1 / 300:  # about one tile in three streams
            s = bytes(rng.choice(alpha) for _ in range(rng.randint(2000, 5000)))
            f = oracle_mod.write_string(s, prefix=7, choice=1)
            longs[k] = oracle_mod.read_string(f, prefix=7)
            kind.append(-1)
            blk += f
        else:
            j = rng.randrange(len(palette))
            kind.append(j)
            blk += palette[j]
    blk = bytes(blk)
    assert len(longs) > 100
    vals, st, nxt = codec.read_strings(blk, pos, [7] * n)
    st, nxt = np.asarray(st), np.asarray(nxt, dtype=np.uint64)
    bad = []
    for i in range(n):
        ref, rc, used = longs[i] if kind[i] < 0 else expect[kind[i]]
        if (vals[i], int(st[i])) != (ref, _oracle_status(rc)) or int(nxt[i]) != pos[i] + used:
            bad.append(i)
    assert not bad, (len(bad), bad[:10])


@pytest.mark.parametrize("order", ["block", "shuffled", "overlap"])
def test_read_random_bytes_as_frames(codec, oracle_mod, order):
    """Random octets read as frames at increasing positions: each string's
    limit at or before the next one's pos (block order: the one-pass read),
    the same strings shuffled (the one-launch fallback, regions back to back),
    or random limits past the next pos (overlapping payloads: the fallback,
    and regions past the output buffer come back NOSPACE) -- every other
    string against the oracle's ReadString over [pos, limit)."""
    NOSPACE = 3
    rng = random.Random({"block": 51, "shuffled": 52, "overlap": 53}[order])
    n = 30000
    blk = bytes(rng.randrange(256) for _ in range(n * 12))
    pos = sorted(rng.randrange(len(blk)) for _ in range(n))
    nxt_pos = pos[1:] + [len(blk)]
    lim = [min(p + rng.randrange(1, 200), len(blk) if order == "overlap" else q) for p, q in zip(pos, nxt_pos)]
    pf = [rng.choice([7, 7, 5, 3, 1]) for _ in range(n)]
    idx = list(range(n))
    if order == "shuffled":
        rng.shuffle(idx)
    P, L, F = [pos[i] for i in idx], [lim[i] for i in idx], [pf[i] for i in idx]
    vals, st, nxt = codec.read_strings(blk, P, F, L)
    checked = 0
    for k in range(n):
        ref, rc, used = oracle_mod.read_string(blk[P[k]:L[k]], prefix=F[k], skip_bits=7 - F[k])
        assert int(nxt[k]) == P[k] + used, (order, k)
        if order == "overlap" and int(st[k]) == NOSPACE:
            continue
        assert (vals[k], int(st[k])) == (ref, _oracle_status(rc)), (order, k)
        checked += 1
    assert checked == n or (order == "overlap" and checked > 1000)


def test_read_wild_pos_and_reverse_order_at_buffer_end(codec, oracle_mod):
    """strings read in reverse block order and header-error
    strings whose pos lies far past the block, with the block ending exactly
    at the end of a 2 MiB device allocation.  The decode must never load from
    blk + pos of an unreadable string, nor prefetch a tile from a reversed
    range; every string against the oracle's ReadString."""
    import numpy as np
    import torch

    rng = random.Random(41)
    strs = _random_strings(rng, 3000)
    blk = b"".join(oracle_mod.write_string(s, prefix=7, choice=1) for s in strs)
    pos, p = [], 0
    for s in strs:
        pos.append(p)
        p += len(oracle_mod.write_string(s, prefix=7, choice=1))
    L = len(blk)
    wild = [L, L + 3, L + 4096, 1 << 33, (1 << 62) + 5]
    P = list(reversed(pos))
    for k, w in enumerate(wild):  # scattered through the reversed run
        P.insert(37 * (k + 1) % len(P), w)
    n = len(P)
    dev = torch.device("cuda:0")
    whole = torch.zeros(2 << 20, dtype=torch.uint8, device=dev)
    t_blk = whole[(2 << 20) - L:]
    t_blk.copy_(torch.frombuffer(bytearray(blk), dtype=torch.uint8).to(dev))
    t_pos = torch.tensor(np.asarray(P, dtype=np.uint64).view(np.int64), device=dev)
    t_lim = torch.full((n,), L, dtype=torch.int64, device=dev)
    t_pf = torch.full((n,), 7, dtype=torch.uint8, device=dev)
    cap = L * 8 // 5 + 16
    out = torch.zeros(cap, dtype=torch.uint8, device=dev)
    out_off = torch.zeros(n + 1, dtype=torch.int64, device=dev)
    out_len = torch.zeros(n, dtype=torch.int32, device=dev)
    st = torch.zeros(n, dtype=torch.uint8, device=dev)
    nxt = torch.zeros(n, dtype=torch.int64, device=dev)
    codec.read_strings_dev(t_blk, t_pos, t_lim, t_pf, out, out_off, out_len, st, nxt)
    torch.cuda.synchronize()
    o = out.cpu().numpy()
    oo = out_off.cpu().numpy().view(np.uint64)
    ol = out_len.cpu().numpy()
    s_h = st.cpu().numpy()
    nx = nxt.cpu().numpy().view(np.uint64)
    for k, q in enumerate(P):
        ref, rc, used = oracle_mod.read_string(blk[q:] if q < L else b"", prefix=7)
        got = o[int(oo[k]): int(oo[k]) + int(ol[k])].tobytes()
        assert (got, int(s_h[k])) == (ref, _oracle_status(rc)), (k, q)
        assert int(nx[k]) == q + used, (k, q)


@pytest.mark.gpu
@pytest.mark.parametrize("order", ["block", "reversed"])
def test_read_regions_layout(codec, oracle_mod, order):
    """The output regions of mhq_read_strings_dev: in block order each starts
    at floor(8*start/5) of its payload start (no scan) and out_off[n] =
    floor(8*blk_len/5); out of block order they lie back to back, each of
    the string's capacity.  Either way disjoint, in string order, and every
    string equals the oracle's."""
    import numpy as np
    import torch

    rng = random.Random(77 if order == "block" else 78)
    strs = _random_strings(rng, 5000)
    blk, pos = bytearray(), []
    for s in strs:
        if rng.random() < 0.3:
            blk += b"\x82"  # another instruction's octet between two fields
        pos.append(len(blk))
        blk += oracle_mod.write_string(s, prefix=7, choice=rng.choice([1, 1, 2]))
    blk = bytes(blk)
    P = pos if order == "block" else list(reversed(pos))
    n, L = len(P), len(blk)
    dev = torch.device("cuda:0")
    t_blk = torch.frombuffer(bytearray(blk), dtype=torch.uint8).to(dev)
    t_pos = torch.tensor(np.asarray(P, dtype=np.int64), device=dev)
    t_lim = torch.full((n,), L, dtype=torch.int64, device=dev)
    t_pf = torch.full((n,), 7, dtype=torch.uint8, device=dev)
    out = torch.zeros(L * 8 // 5 + 16, dtype=torch.uint8, device=dev)
    out_off = torch.zeros(n + 1, dtype=torch.int64, device=dev)
    out_len = torch.zeros(n, dtype=torch.int32, device=dev)
    st = torch.zeros(n, dtype=torch.uint8, device=dev)
    nxt = torch.zeros(n, dtype=torch.int64, device=dev)
    codec.read_strings_dev(t_blk, t_pos, t_lim, t_pf, out, out_off, out_len, st, nxt)
    torch.cuda.synchronize()
    o, oo, ol = out.cpu().numpy(), out_off.cpu().numpy(), out_len.cpu().numpy()
    assert (np.diff(oo) >= 0).all()
    for k, q in enumerate(P):
        ref, rc, used = oracle_mod.read_string(blk[q:], prefix=7)
        assert o[oo[k]:oo[k] + ol[k]].tobytes() == ref and int(st[k]) == _oracle_status(rc), k
        assert int(nxt[k]) == q + used
        take, _, hdr = oracle_mod.read_int(blk[q:], 7, skip_bits=1)
        start = q + hdr
        cap = take * 8 // 5 if blk[q] & 0x80 else take
        if order == "block":
            assert oo[k] == start * 8 // 5, k
        assert oo[k] + cap <= oo[k + 1], k
        if order != "block":
            assert oo[k + 1] - oo[k] == cap, k
    if order == "block":
        assert oo[n] == L * 8 // 5


@pytest.mark.parametrize("order", ["in_order", "runs"])
def test_read_poisoned_scratch(codec, oracle_mod, monkeypatch, order):
    """Stale scratch that matches the call's flags in their round-4 form
    (mhq_debug_poison_scratch, str_frame.hip): a fallback word whose LOW word
    equals the call's generation number -- round 4's fused pass compared only
    that and stopped its waves, while the fallback, comparing all 64 bits, did
    nothing: strings left unwritten -- and look-back slots carrying round 4's
    tag of the call with garbage sums -- its fallback added those up: regions
    laid out wrong.  2^19 strings, so every wave of the fused pass has two
    tiles; in block order (the fused pass alone) and in shuffled runs of 300
    (the fallback, 255 workgroups looking back).  The device outputs start as
    sentinels; every string equals the host call's result (unpoisoned), and a
    sample the oracle's."""
    import numpy as np
    import torch

    rng = random.Random(36 if order == "in_order" else 37)
    alpha = b"abcdefghijklmnopqrstuvwxyz0123456789-_./:;=, "
    n = 1 << 19
    pieces = [oracle_mod.write_string(bytes(rng.choice(alpha) for _ in range(rng.randint(0, 40))), prefix=7,
                                      choice=rng.choice([1, 1, 1, 2])) for _ in range(4096)]
    blk, pos = bytearray(), []
    for _ in range(n):
        pos.append(len(blk))
        blk += pieces[rng.randrange(len(pieces))]
    blk = bytes(blk)
    if order == "runs":
        runs = [pos[k:k + 300] for k in range(0, n, 300)]
        rng.shuffle(runs)
        pos = [p for r in runs for p in r]
    ref_vals, ref_st, ref_nxt = codec.read_strings(blk, pos, [7] * n)
    L = len(blk)
    dev = torch.device("cuda:0")
    t_blk = torch.frombuffer(bytearray(blk), dtype=torch.uint8).to(dev)
    t_pos = torch.tensor(np.asarray(pos, dtype=np.int64), device=dev)
    t_lim = torch.full((n,), L, dtype=torch.int64, device=dev)
    t_pf = torch.full((n,), 7, dtype=torch.uint8, device=dev)
    out = torch.full((L * 8 // 5 + 16,), 0xA5, dtype=torch.uint8, device=dev)
    out_off = torch.full((n + 1,), -1, dtype=torch.int64, device=dev)
    out_len = torch.full((n,), -1, dtype=torch.int32, device=dev)
    st = torch.full((n,), 0xEE, dtype=torch.uint8, device=dev)
    nxt = torch.full((n,), -1, dtype=torch.int64, device=dev)
    codec._L.mhq_debug_poison_scratch(1)
    try:
        codec.read_strings_dev(t_blk, t_pos, t_lim, t_pf, out, out_off, out_len, st, nxt)
        torch.cuda.synchronize()
    finally:
        codec._L.mhq_debug_poison_scratch(0)
    oo = out_off.cpu().numpy().view(np.uint64)
    ol = out_len.cpu().numpy().view(np.uint32)
    assert (st.cpu().numpy() == np.asarray(ref_st)).all()
    assert (nxt.cpu().numpy().view(np.uint64) == np.asarray(ref_nxt)).all()
    assert (ol == np.asarray([len(v) for v in ref_vals], dtype=np.uint32)).all()
    assert int(oo[n]) <= out.numel() and (np.diff(oo.astype(np.int64)) >= 0).all()
    o = out.cpu().numpy()
    assert all(o[int(oo[k]): int(oo[k]) + int(ol[k])].tobytes() == ref_vals[k] for k in range(n))
    for i in sorted(rng.sample(range(n), 5000)):
        ref, rc, used = oracle_mod.read_string(blk[pos[i]:pos[i] + 200], prefix=7)
        assert (ref_vals[i], int(ref_st[i])) == (ref, _oracle_status(rc)), i
        assert int(ref_nxt[i]) == pos[i] + used
