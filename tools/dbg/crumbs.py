"""Reads a mhq_dbg_crumbs_dump file (-DMHQ_DBG_CRUMBS build, read_strings.hip):
per lane of read_fused_kernel the last (site, address) before a global
access; prints the lanes whose address lies outside every buffer of the call."""
import sys

import numpy as np

d = np.fromfile(sys.argv[1], dtype=np.uint64)
h = d[:24]
lanes = int(h[1])
blk, blk_len, pos, limit, prefix, n, out, out_off, nxt, out_len, status, sc_start, sc_hend, sc_kind, fb, wg_agg, gen, grid, per_block, tl = (int(x) for x in h[2:22])
nout = blk_len // 5 * 8 + (blk_len % 5) * 8 // 5
bufs = {"blk": (blk, blk_len), "pos": (pos, 8 * n), "limit": (limit, 8 * n), "prefix": (prefix, n),
        "out": (out, nout + 1), "out_off": (out_off, 8 * (n + 1)), "next": (nxt, 8 * n), "out_len": (out_len, 4 * n),
        "status": (status, n), "sc_start": (sc_start, 8 * (n + 1)), "sc_hend": (sc_hend, 4 * (n + 1)),
        "sc_kind": (sc_kind, n + 1), "fallback": (fb, 8), "wg_agg": (wg_agg, 8 * 4096)}
print(f"n={n} blk_len={blk_len} grid={grid} per_block={per_block} tl={tl} gen={gen}")
for k, (b, sz) in bufs.items():
    print(f"  {k:9s} {b:#x} .. {b + sz:#x}")
c = d[24:24 + 2 * lanes].reshape(-1, 2)
live = np.nonzero(c[:, 0])[0]
sites = {}
bad = []
for i in live:
    site, addr = int(c[i, 0]), int(c[i, 1])
    sites[site] = sites.get(site, 0) + 1
    hit = [k for k, (b, sz) in bufs.items() if b <= addr < b + sz]
    if not hit:
        near = min(bufs.items(), key=lambda kv: min(abs(addr - kv[1][0]), abs(addr - kv[1][0] - kv[1][1])))
        bad.append((i, site, addr, near[0], addr - near[1][0]))
print("last sites (site: lanes):", dict(sorted(sites.items())))
print(f"{len(bad)} lanes outside every buffer")
for i, site, addr, k, off in bad[:60]:
    print(f"  wg {i // 768} wave {(i % 768) // 64} lane {i % 64}: site {site} addr {addr:#x} ({k}{off:+d})")
