// read_strings.hip -- gfx950 batch Reader.ReadString (hc/io.go:73-97) in one
// pass: the framing parse inside the decode's tile staging, plus the
// one-launch fallback for strings out of block order.  The decode core is
// huff_decode_dev.h.
#include <hip/hip_runtime.h>

#include "huff_decode_dev.h"

#ifdef MHQ_DBG_CRUMBS
#include <algorithm>
#include <cstdio>
#include <cstring>
#endif

namespace mhq {
namespace {

using namespace dev;

// ---- read_strings in one pass (MHQ_RS_FUSED) -----------------------------
// Reader.ReadString over a batch of framed strings (hc/io.go:73-97, 25-55),
// each tile's frames parsed from its staged bytes: a tile is the byte span
// [pos[s], pos[s + cnt]) of its strings, staged as the in_end decode stages
// the payloads alone, so the parse costs no extra pass over HBM (the
// multi-pass pipeline reads pos / limit / prefix and the headers, writes
// start / hend / kind, and the decode reads those back).  Output regions are
// the positional layout, string i's at floor(8 start_i / 5) (str_frame.hip):
// a tile's regions lie in [floor(8 pos[s] / 5), floor(8 pos[s + cnt] / 5)).
// A tile over the slices parses from global memory into sc_* and streams
// (decode_tile_long).  Strings out of block order -- or a header integer that
// runs past the next string's pos -- store gen to *fallback and the tile is
// left: the caller's gated passes then redo the whole call.
struct RsArgs {
  const uint8_t *blk;
  uint64_t blk_len;
  const uint64_t *pos, *limit;
  const uint8_t *prefix;
  uint64_t n;
  uint8_t *out;
  uint64_t *out_off, *next;
  uint32_t *out_len;
  uint8_t *status;
  uint64_t *sc_start;
  uint32_t *sc_hend;
  uint8_t *sc_kind;
  uint64_t *fallback;
  uint64_t gen;
  uint64_t *wg_agg;  // the fallback's look-back slots: cleared here (workgroup 0), kReadFallbackMaxWgs words
};

struct RsTile {  // pos / limit / prefix of strings s + 2 lane + {0, 1}; pos of string s + tile
  uint64_t p0, p1, l0, l1, pe;
  uint32_t pf;  // prefix of the first | of the second << 8
};

__device__ __forceinline__ void rs_load(RsTile &t, const RsArgs &a, uint64_t s, uint64_t L1, uint32_t tl,
                                        uint32_t lane) {
  const uint32_t z = vzero();
  const uint64_t j0 = min(s + 2u * lane, L1 - 1u) + z, j1 = min(s + 2u * lane + 1u, L1 - 1u) + z;
  CRUMB(1, a.limit + j1);
  CRUMB(2, a.prefix + j1);
  CRUMB(3, a.pos + min(min(s + (uint64_t)tl, L1), a.n - 1u));
  t.p0 = a.pos[j0];
  t.p1 = a.pos[j1];
  t.l0 = a.limit[j0];
  t.l1 = a.limit[j1];
  t.pf = (uint32_t)a.prefix[j0] | (uint32_t)a.prefix[j1] << 8;
  t.pe = a.pos[min(min(s + (uint64_t)tl, L1), a.n - 1u) + z];  // (used only below n)
}

struct RsStr {
  uint64_t start, take;
  uint32_t kind;  // 0 raw, 1 Huffman, 2 header error; | kDeclared
  bool far;       // a header octet outside [lo, hi): not read
};

// Reader.ReadBit + ReadInt(prefix) of the frame at p, reading no octet at or
// past lim (the read_parse_kernel rules, str_frame.hip), octets by `byte`.
template <class Byte>
__device__ __forceinline__ RsStr rs_parse(uint64_t p, uint64_t lim, uint32_t pf, uint64_t blk_len, uint64_t lo,
                                          uint64_t hi, Byte byte) {
  RsStr r{p < blk_len ? p : blk_len, 0, 2u, false};
  if (pf < 1u || pf > 7u || p >= lim) return r;
  if (p < lo || p >= hi) {
    r.far = true;
    return r;
  }
  const uint32_t b0 = byte(p);
  const uint64_t mask = (1ull << pf) - 1u;
  uint64_t v = b0 & mask, q = p + 1;
  if (v == mask) {
    for (uint32_t sh = 0; sh < 64; sh += 7) {
      if (q >= lim) return r;  // EOF inside the integer
      if (q >= hi) {
        r.far = true;
        return r;
      }
      const uint64_t b = byte(q++);
      if (sh == 63 && (b > 1 || (b == 1 && (v >> 63) == 1))) return r;  // ErrIntegerOverflow (hc/io.go:46)
      v += (b & 0x7f) << sh;
      if ((b & 0x80) == 0) break;
    }
  }
  r.kind = ((b0 >> pf) & 1u) | (v != 0 ? kDeclared : 0u);
  r.start = q;
  r.take = min(v, lim - q);
  return r;
}

// Octet x of the staged input slice (words byte-swapped by put_chunk).
__device__ __forceinline__ uint32_t slice_byte(const WaveSmem &ws, uint32_t x) {
  return (ws.in_w[x >> 2] >> (24u - 8u * (x & 3u))) & 0xffu;
}

// out_len / status of strings [s, s + m): ReadString's outcome by kind
// (hc/io.go:92-96); `kinds` holds string 2 l + h's kind at bits 4h of lane l.
__device__ __forceinline__ void flush_str(const WaveSmem &ws, uint64_t s, uint32_t m, uint32_t kinds,
                                          uint32_t *__restrict__ out_len, uint8_t *__restrict__ status,
                                          uint32_t lane) {
#pragma unroll
  for (int h = 0; h < 2; h++) {
    const uint32_t j = lane + (uint32_t)kWave * h;
    const uint32_t kd = ((uint32_t)__shfl((int)kinds, (int)(j >> 1)) >> (4u * (j & 1u))) & 7u;
    if (j < m) {
      const uint32_t v = ws.len[j];
      uint32_t len = v & 0x7fffffffu, st = v >> 31;
      if ((kd & 3u) == 1u) {  // Huffman: INVALID keeps 0 bytes, nothing decoded is io.EOF
        if (st) len = 0;
        else if (len == 0) st = kStrEof;
      } else if ((kd & 3u) == 0u) {  // raw: len is the payload copied
        st = len == 0 && (kd & kDeclared) ? kStrEof : 0u;
      } else {  // ReadBit / ReadInt failed: ("", nil)
        len = 0;
        st = 0;
      }
      CRUMB(4, status + s + j);
      __builtin_nontemporal_store(len, out_len + s + j);
      __builtin_nontemporal_store((uint8_t)st, status + s + j);
    }
  }
}

__global__ __launch_bounds__(kT) void read_fused_kernel(RsArgs a, const uint32_t *__restrict__ g_lut1,
                                                        const uint16_t *__restrict__ g_lut2,
                                                        const uint8_t *__restrict__ g_len, uint64_t per_block,
                                                        uint32_t tl) {
  __shared__ Smem sm;
  const uint32_t tid = threadIdx.x;
  const uint32_t lane = tid % kWave;
  const uint32_t wave = tid / kWave;
  const uint64_t L0 = (uint64_t)blockIdx.x * per_block;
  if (L0 >= a.n) return;
  const uint64_t L1 = min(L0 + per_block, a.n);
  WaveSmem &ws = sm.w[wave];
  const uint64_t blk_len = a.blk_len;
  // the fallback's look-back slots start every call cleared (stream order
  // puts this before the fallback launch): a slot then holds this call's tag
  // or 0, never stale data -- the per-stream scratch is shared with other
  // calls and entry points, whose words could otherwise carry a matching tag
  if (blockIdx.x == 0)
    for (uint32_t g = tid; g < kReadFallbackMaxWgs; g += kT) a.wg_agg[g] = 0;
  // a tile's byte span, clamped to the block (empty past the range)
  auto span = [&](const RsTile &t, uint64_t s, uint64_t &ps, uint64_t &pe) {
    ps = pe = 0;
    if (s >= L1) return;
    const uint64_t e = min(s + (uint64_t)tl, L1);
    ps = min(uniform64(t.p0), blk_len);
    pe = e < a.n ? min(uniform64(t.pe), blk_len) : blk_len;
  };
  uint32_t tile = wave, tile2 = tile + kWaves, tile3 = tile + 2 * kWaves;
  RsTile rt, rn;
  rs_load(rt, a, L0 + (uint64_t)tile * tl, L1, tl, lane);
  TileIn tin;
  uint32_t keep[kPF] = {};
  {
    uint64_t ps, pe;
    span(rt, L0 + (uint64_t)tile * tl, ps, pe);
    load_in(tin, a.blk, 0, ps, pe, lane, keep);
  }
  static_assert(kLut1Size / 4 <= 2 * kT && kLut2Size / 8 <= kT && kT >= 64, "table copy shape");
  const uint32_t x1 = min(tid + (uint32_t)kT, (uint32_t)(kLut1Size / 4) - 1u);
  const uint32_t x2 = min(tid, (uint32_t)(kLut2Size / 8) - 1u), x3 = tid % 64u;
  const u32x4 tb0 = ((const u32x4 *)g_lut1)[tid];
  const u32x4 tb1 = ((const u32x4 *)g_lut1)[x1];
  const u32x4 tb2 = ((const u32x4 *)g_lut2)[x2];
  const uint32_t tb3 = ((const uint32_t *)g_len)[x3];
  rs_load(rn, a, L0 + (uint64_t)tile2 * tl, L1, tl, lane);
  ((u32x4 *)sm.lut1)[tid] = tb0;
  ((u32x4 *)sm.lut1)[x1] = tb1;
  ((u32x4 *)sm.lut2)[x2] = tb2;
  ((uint32_t *)sm.clen)[x3] = tb3;
  if (tid == 0) sm.next_tile = 3 * kWaves;
  __syncthreads();
#pragma unroll
  for (int k = 0; k < kPF; k++) asm volatile("" ::"v"(keep[k]));
  const uint32_t ntiles = (uint32_t)((L1 - L0 + tl - 1) / tl);
  uint64_t pd_s = 0;  // the previous tile, still in the output slice
  uint32_t pd_m = 0, pd_lo = 0, pd_hi = 0, kinds = 0;
  uint8_t *pd_o = nullptr;
  uint32_t tl_j = 0;
  // the fallback word, loaded a tile ahead: a wave stops once some wave has
  // sent the call to the fallback (the whole word is compared: the scratch
  // holds stale data, whose low word may well equal a small gen counter)
  uint64_t fb_seen = 0;

  while (tile < ntiles) {
    if (uniform64(fb_seen) == a.gen) break;
    const uint64_t s = L0 + (uint64_t)tile * tl;
    const uint32_t cnt = (uint32_t)min((uint64_t)tl, L1 - s);
    uint64_t ps, pe;
    span(rt, s, ps, pe);
    const uint8_t *ia = a.blk + ps;
    const uint64_t rs0 = region_at(ps), rs1 = region_at(pe);
    uint8_t *oa = a.out + rs0;
    const uint32_t idelta = (uint32_t)((uintptr_t)ia & 15u), odelta = (uint32_t)((uintptr_t)oa & 15u);
    bool fits = pe >= ps && (pe - ps) + idelta <= (uint64_t)kWIn && (rs1 - rs0) + odelta <= (uint64_t)kWOut;
    DBG_CHECK(!fits || rs1 <= region_at(blk_len), 10, rs1, blk_len);
    __builtin_amdgcn_s_setprio(kPhasePrio);
    uint32_t tile4 = 0;
    if (lane == 0) tile4 = atomicAdd(&sm.next_tile, 1u);
    if (fits) {
      const uint32_t chunks = (uint32_t)(((pe - ps) + idelta + 15u) >> 4);
#pragma unroll
      for (int k = 0; k < kPF; k++) {
        const uint32_t c = lane + (uint32_t)kWave * k;
        if (c < chunks) put_chunk(ws, c, tin.v[k]);
      }
    }
    // the previous tile's output and lengths leave (its kinds are read here,
    // before this tile's parse replaces them)
    if (pd_o) {
      if (DBG_OK(dbg_out_ok(pd_o + pd_lo, pd_hi - pd_lo), 34, pd_o, pd_hi))
        store_out_batched<kOutRounds>(pd_o, (const uint8_t *)ws.out_w, pd_lo, pd_hi, lane);
      flush_str(ws, pd_s, pd_m, kinds, a.out_len, a.status, lane);
    }
    pd_o = nullptr;
    wave_sync();
    // the frames: from the slice when staged, else from global memory
    const uint64_t lo = fits ? ps : 0, hi = fits ? pe : blk_len;
    uint32_t raw0 = 0, raw1 = 0;  // raw payload lengths
    bool bad = false;
    kinds = 0;
#pragma unroll
    for (int h = 0; h < 2; h++) {
      const uint32_t j = 2u * lane + (uint32_t)h;
      const uint64_t nx = (uint64_t)__shfl_down((unsigned long long)rt.p0, 1);
      if (j < cnt) {
        const uint64_t p = h ? rt.p1 : rt.p0;
        const uint64_t lim = min(h ? rt.l1 : rt.l0, blk_len);
        const uint32_t pf = (rt.pf >> (8 * h)) & 0xffu;
        const uint64_t pn = j + 1u < cnt ? (h ? nx : rt.p1) : pe;  // the next string's pos (order test)
        RsStr r = rs_parse(p, lim, pf, blk_len, lo, hi, [&](uint64_t q) -> uint32_t {
          if (!fits) CRUMB(5, a.blk + q);
          return fits ? slice_byte(ws, (uint32_t)(q - ps) + idelta) : (uint32_t)a.blk[q];
        });
        if (r.far)  // a header octet outside the staged span: from global memory (bad below unless it failed)
          r = rs_parse(p, lim, pf, blk_len, 0, blk_len, [&](uint64_t q) -> uint32_t {
            CRUMB(6, a.blk + q);
            return a.blk[q];
          });
        bad |= r.start + r.take > min(pn, blk_len);  // read_parse_kernel's order test
        const uint32_t k = r.kind & 3u;
        const uint64_t hend = k == 1u ? r.start + r.take : r.start;
        const uint64_t reg = region_at(r.start), i = s + j;
        kinds |= r.kind << (4 * h);
        if (k == 0u) (h ? raw1 : raw0) = (uint32_t)r.take;
        CRUMB(7, a.next + i);
        a.out_off[i] = reg;  // (streaming stores: 1.6 us slower)
        a.next[i] = k == 2u ? p : r.start + r.take;
        if (fits) {
          ws.rec[j] = (uint32_t)(r.start - ps + idelta) | (uint32_t)(reg - rs0 + odelta) << 16;
          ws.len[j] = (uint32_t)(hend - ps + idelta);
        } else {
          CRUMB(8, a.sc_kind + i);
          a.sc_start[i] = r.start;
          a.sc_hend[i] = (uint32_t)hend;
          a.sc_kind[i] = (uint8_t)r.kind;
        }
      }
    }
    if (lane == 0 && s + cnt == a.n) a.out_off[a.n] = region_at(blk_len);
    const bool skip = __ballot(bad) != 0;  // (uniform)
    if (skip && lane == 0) *a.fallback = a.gen;  // (every writer stores the same value)
    if (fits && lane == 0) ws.rec[cnt] = (uint32_t)(pe - ps + idelta) | (uint32_t)(rs1 - rs0 + odelta) << 16;
    wave_sync();
    // the next tile's input, the frames of the one after
    {
      uint64_t ps2, pe2;
      span(rn, L0 + (uint64_t)tile2 * tl, ps2, pe2);
      load_in(tin, a.blk, 0, ps2, pe2, lane);
    }
    fb_seen = __builtin_nontemporal_load(a.fallback + vzero());  // (after the input loads: waited for with them)
    rt = rn;
    rs_load(rn, a, L0 + (uint64_t)tile3 * tl, L1, tl, lane);
    if (skip) {
    } else if (fits) {
      const uint32_t out_bytes = (uint32_t)(rs1 - rs0) + odelta;
#ifdef MHQ_DBG_BOUNDS
      for (uint32_t j = lane; j < cnt; j += kWave)
        DBG_CHECK((ws.rec[j] & 0xffffu) <= ws.len[j] && ws.len[j] <= (uint32_t)(pe - ps) + idelta &&
                      (ws.rec[j] >> 16) <= (ws.rec[j + 1] >> 16),
                  11, ws.rec[j] | (uint64_t)ws.rec[j + 1] << 32, ws.len[j] | (uint64_t)(pe - ps + idelta) << 32);
#endif
      decode_piece<true>(sm, ws, cnt, out_bytes, lane, -1, tl_j < 2u ? 1u : 0u);
      // raw payloads into their regions
#pragma unroll
      for (int h = 0; h < 2; h++) {
        const uint32_t j = 2u * lane + (uint32_t)h, take = h ? raw1 : raw0;
        if (j < cnt && ((kinds >> (4 * h)) & 3u) == 0u) {
          const uint32_t r = ws.rec[j], x = r & 0xffffu, y = r >> 16;
          DBG_CHECK(y + take <= out_bytes && x + take <= (uint32_t)(pe - ps) + idelta, 14, y + take, x + take);
          uint8_t *o = (uint8_t *)ws.out_w;
          for (uint32_t k = 0; k < take; k++) o[y + k] = (uint8_t)slice_byte(ws, x + k);
          ws.len[j] = take;
        }
      }
      wave_sync();
      pd_o = oa - odelta;
      pd_lo = odelta;
      pd_hi = out_bytes;
      pd_s = s;
      pd_m = cnt;
    } else {
      // streamed: out_off[s + cnt] (the last region's end) from the next
      // string's frame, then the long-literal decode over sc_*
      // (every lane parses the same frame -- uniform control flow, scalar
      // loads -- and lane 0 stores: a lane-0-only block here is where the
      // register allocator put the copies and spill stores of values live
      // across the old call, with the other 63 lanes masked off; DESIGN.md,
      // round 6)
      if (s + cnt < a.n) {
        const uint64_t i = s + cnt;
        CRUMB(9, a.out_off + i);
        const RsStr r = rs_parse(a.pos[i], min(a.limit[i], blk_len), a.prefix[i], blk_len, 0, blk_len,
                                 [&](uint64_t q) -> uint32_t {
                                   CRUMB(10, a.blk + q);
                                   return a.blk[q];
                                 });
        if (lane == 0) a.out_off[i] = region_at(r.start);
      }
      __threadfence_block();
      wave_sync();
      decode_tile_long_body<true>(sm, ws, a.blk, a.sc_start, a.sc_hend, 0, a.out, a.out_off, 0, a.out_len, a.status,
                                  s, cnt, lane, a.sc_kind);
      __threadfence_block();
      for (uint32_t j = lane; j < cnt; j += kWave) {  // the lane that wrote string j's length
        const uint64_t i = s + j;
        CRUMB(11, a.next + i);
        const uint8_t kd = a.sc_kind[i];
        if ((kd & 3u) != 0u) continue;
        const uint64_t st0 = a.sc_start[i], take = a.next[i] - st0;
        if (take) {
          DBG_CHECK(a.out_off[i] + take <= region_at(blk_len) && st0 + take <= blk_len, 12, a.out_off[i], take);
          if (DBG_OK(dbg_out_ok(a.out + a.out_off[i], take) && dbg_in_ok(a.blk + st0, take), 33, a.out_off[i], take))
            copy_bytes(a.out + a.out_off[i], a.blk + st0, take);
          a.out_len[i] = (uint32_t)take;
        } else if (kd & kDeclared) {
          a.status[i] = (uint8_t)kStrEof;  // the block ended before the payload: io.EOF
        }
      }
      wave_sync();
    }
    tl_j++;
    tile = tile2;
    tile2 = tile3;
    tile3 = __builtin_amdgcn_readfirstlane(tile4);
  }
  if (pd_o) {
    if (DBG_OK(dbg_out_ok(pd_o + pd_lo, pd_hi - pd_lo), 34, pd_o, pd_hi))
      store_out_batched<kOutRounds>(pd_o, (const uint8_t *)ws.out_w, pd_lo, pd_hi, lane);
    flush_str(ws, pd_s, pd_m, kinds, a.out_len, a.status, lane);
  }
}

// ---- the fused read's fallback: strings out of block order, one launch ----
// When read_fused_kernel stored gen to *fallback (some string's payload runs
// past the next string's pos: the strings are out of block order), this
// kernel redoes the call as read_parse_kernel -> the capacities scan ->
// decode_kernel<true> would (str_frame.hip) for out-of-order strings: regions
// back to back, clamped to out_cap.  Each workgroup parses its decode range
// (and the string after it, whose payload start bounds its last tile),
// publishes its capacity sum, adds up its predecessors' sums as they appear
// (decoupled look-back: every predecessor publishes right after its own
// parse, so one round usually sees them all), lays out its regions and
// decodes its range with the range's own bounds (StrFinish::local).  No
// workgroup reads another's data except the published sums (agent-scope
// atomics): no grid barrier, no device-wide fence, and a workgroup only ever
// waits for lower-numbered ones, which the dispatcher started first -- no
// assumption that the grid is resident at once.  In block order every
// workgroup returns at once: one launch instead of three gated ones (6.4 us
// of the call on the config-2 block).
struct RsFallback {
  RsArgs a;
  uint64_t out_cap;
  uint64_t *wg_agg;  // per workgroup: agg_tag(gen) | capacity sum (0 until published; cleared by the fused pass)
  uint64_t *wg_fin;  // per workgroup: gen when its range holds a raw string
  uint32_t help_polls;  // polls of a predecessor's sum before it is computed here (see the look-back)
};
constexpr uint64_t kAggBits = 40;  // a workgroup's capacity sum < 2^40
// A published sum's tag: 23 bits of the call's generation number and a set
// bit, never 0, so a cleared slot never matches (and the read_fused_kernel
// clears every slot before this launch).
__device__ __forceinline__ uint64_t agg_tag(uint64_t gen) { return ((gen & 0x7fffffull) | 0x800000ull) << kAggBits; }

// The capacity sum workgroup g publishes (its strings [L0, L1)), computed
// by one thread from the frames in global memory: the look-back's way out
// when g stays unpublished -- the dispatcher starts workgroups in order per
// XCD, not across the chip, so with concurrent launches g may be waiting for
// a slot that polling workgroups hold.
__device__ __forceinline__ uint64_t range_cap_sum(const RsArgs &a, uint64_t L0, uint64_t L1) {
  uint64_t csum = 0;
  for (uint64_t i = L0; i < L1; i++) {
    const RsStr r = rs_parse(a.pos[i], min(a.limit[i], a.blk_len), a.prefix[i], a.blk_len, 0, a.blk_len,
                             [&](uint64_t q) -> uint32_t { return a.blk[q]; });
    const uint32_t k = r.kind & 3u;
    csum += k == 1u ? r.take * 8u / 5u : (k == 0u ? r.take : 0u);
  }
  return csum;
}

// Sum of v over the workgroup (every thread gets it); red: kWaves words.
__device__ __forceinline__ uint64_t wg_sum(uint64_t v, uint64_t *red) {
#pragma unroll
  for (int d = 1; d < kWave; d <<= 1) v += __shfl_xor((unsigned long long)v, d);
  if (threadIdx.x % kWave == 0) red[threadIdx.x / kWave] = v;
  __syncthreads();
  uint64_t t = 0;
#pragma unroll
  for (int w = 0; w < kWaves; w++) t += red[w];
  __syncthreads();
  return t;
}

__global__ __launch_bounds__(kT) void read_fallback_kernel(RsFallback f, const uint32_t *__restrict__ g_lut1,
                                                           const uint16_t *__restrict__ g_lut2,
                                                           const uint8_t *__restrict__ g_len, uint64_t per_block,
                                                           uint32_t tl0) {
  __shared__ Smem sm;
  __shared__ uint64_t red[kWaves];
  const RsArgs &a = f.a;
  if (__builtin_nontemporal_load(a.fallback) != a.gen) return;  // (the whole grid alike)
  const uint32_t tid = threadIdx.x, b = blockIdx.x;
  const uint64_t n = a.n, blk_len = a.blk_len;
  const uint64_t L0 = (uint64_t)b * per_block, L1 = min(L0 + per_block, n);
  const uint64_t tag = agg_tag(a.gen);
  // parse (read_parse_kernel's rules, str_frame.hip) of [L0, L1] -- string L1
  // too (its payload start is in_off[L1], read by this range's last tile; its
  // own workgroup writes the same value)
  uint64_t csum = 0;
  bool raw = false;
  for (uint64_t i = L0 + tid; i <= L1; i += kT) {
    if (i == n) {
      a.sc_start[n] = blk_len;
      break;
    }
    const RsStr r = rs_parse(a.pos[i], min(a.limit[i], blk_len), a.prefix[i], blk_len, 0, blk_len,
                             [&](uint64_t q) -> uint32_t { return a.blk[q]; });
    a.sc_start[i] = r.start;
    if (i == L1) break;
    const uint32_t k = r.kind & 3u;
    a.sc_hend[i] = (uint32_t)(k == 1u ? r.start + r.take : r.start);
    a.sc_kind[i] = (uint8_t)r.kind;
    a.next[i] = k == 2u ? a.pos[i] : r.start + r.take;
    csum += k == 1u ? r.take * 8u / 5u : (k == 0u ? r.take : 0u);
    raw |= k == 0u;
  }
  const bool any_raw = __syncthreads_or(raw);
  if (tid == 0) f.wg_fin[b] = any_raw ? a.gen : 0u;
  const uint64_t total = wg_sum(csum, red);
  if (tid == 0) __hip_atomic_store((unsigned long long *)f.wg_agg + b, tag | total, __ATOMIC_RELAXED,
                                   __HIP_MEMORY_SCOPE_AGENT);
  // look-back: the sums of workgroups 0 .. b-1, each once it carries this
  // call's tag (every thread takes every kT-th predecessor)
  uint64_t base = 0;
  for (uint32_t g0 = 0; g0 < b; g0 += kT) {
    const uint32_t g = g0 + tid;
    uint64_t v = 0;
    if (g < b) {
      for (uint32_t polls = 0;; polls++) {
        v = __hip_atomic_load((unsigned long long *)f.wg_agg + g, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        if ((v & ~((1ull << kAggBits) - 1u)) == tag) break;
        if (polls >= f.help_polls) {  // unpublished too long: its sum from its frames (range_cap_sum)
          v = tag | range_cap_sum(a, (uint64_t)g * per_block, min((uint64_t)g * per_block + per_block, n));
          break;
        }
        __builtin_amdgcn_s_sleep(1);
      }
    }
    base += v & ((1ull << kAggBits) - 1u);
  }
  base = wg_sum(base, red);
  // the regions back to back from base, clamped to out_cap
  for (uint64_t c0 = L0; c0 < L1; c0 += kT) {
    const uint64_t i = c0 + tid;
    const uint64_t cap = i < L1 ? read_cap(a.sc_kind[i], a.sc_start[i], a.sc_hend[i], a.next[i]) : 0u;
    uint64_t x = cap;  // inclusive scan over the wave, then over the waves
#pragma unroll
    for (int d = 1; d < kWave; d <<= 1) {
      const uint64_t y = __shfl_up((unsigned long long)x, d);
      if ((tid % kWave) >= (uint32_t)d) x += y;
    }
    if (tid % kWave == kWave - 1) red[tid / kWave] = x;
    __syncthreads();
    uint64_t before = 0, all = 0;
#pragma unroll
    for (int w = 0; w < kWaves; w++) {
      before += w < (int)(tid / kWave) ? red[w] : 0u;
      all += red[w];
    }
    __syncthreads();
    if (i < L1) a.out_off[i] = min(base + before + x - cap, f.out_cap);
    base += all;
  }
  if (tid == 0) a.out_off[L1] = min(base, f.out_cap);  // (the next workgroup writes the same value)
  __threadfence_block();  // this range's parse and layout, for the decode's other waves
  __syncthreads();
  StrFinish str;
  str.kind = a.sc_kind;
  str.start = a.sc_start;
  str.next = a.next;
  str.hend = a.sc_hend;
  str.blk = a.blk;
  str.out_cap = f.out_cap;
  str.finish_needed = f.wg_fin + b;
  str.gen = a.gen;
  str.local = true;
  decode_body<true>(sm, a.blk, a.sc_start, a.sc_hend, str, 0, n, a.out, a.out_off, 0, a.out_len, a.status, g_lut1,
                    g_lut2, g_len, per_block, tl0);
}

}  // namespace

// The decode's grid and tile length (launch_decode), the tile length cut to
// what fits the slices at the block's mean frame (decode_kernel's kGaps rule).
#ifdef MHQ_DBG_CRUMBS
// -DMHQ_DBG_CRUMBS: read_fused_kernel's lanes leave (site, address) crumbs in
// pinned host memory (huff_common.h); the last launch's arguments are kept
// for mhq_dbg_crumbs_dump.
unsigned long long *g_crumb_host;
uint64_t g_crumb_lanes, g_crumb_geom[3];
RsArgs g_crumb_args;
void crumbs_arm(const RsArgs &a, unsigned grid, uint64_t per_block, uint64_t tl, hipStream_t s) {
  const uint64_t lanes = (uint64_t)std::max<unsigned>(grid, kReadFallbackMaxWgs) * kT;
  (void)hipStreamSynchronize(s);
  if (lanes > g_crumb_lanes) {
    if (g_crumb_host) (void)hipHostFree(g_crumb_host);
    g_crumb_host = nullptr;
    if (hipHostMalloc((void **)&g_crumb_host, lanes * 16, hipHostMallocCoherent | hipHostMallocMapped) != hipSuccess)
      return;
    g_crumb_lanes = lanes;
  }
  memset(g_crumb_host, 0, g_crumb_lanes * 16);
  unsigned long long *d = nullptr;
  (void)hipHostGetDevicePointer((void **)&d, g_crumb_host, 0);
  (void)hipMemcpyToSymbol(HIP_SYMBOL(g_crumbs), &d, sizeof(d));
  g_crumb_args = a;
  g_crumb_geom[0] = grid;
  g_crumb_geom[1] = per_block;
  g_crumb_geom[2] = tl;
}
#endif

hipError_t launch_read_fused(const DevTables &t, const uint8_t *blk, uint64_t blk_len, const uint64_t *pos,
                             const uint64_t *limit, const uint8_t *prefix, uint64_t n, uint8_t *out,
                             uint64_t *out_off, uint32_t *out_len, uint8_t *status, uint64_t *next,
                             uint64_t *sc_start, uint32_t *sc_hend, uint8_t *sc_kind, uint64_t *fallback,
                             uint64_t *wg_agg, uint64_t gen, hipStream_t s) {
  if (n == 0) return hipSuccess;
  const uint64_t cus = (uint64_t)dev::device_cus();
  const uint64_t slots = cus * kWaves;
  const uint64_t rounds = (n + slots * kTile - 1) / (slots * kTile);
  uint64_t tl = std::max<uint64_t>(1, (n + slots * rounds - 1) / (slots * rounds));
  const uint64_t nout = blk_len / 5 * 8 + (blk_len % 5) * 8 / 5;
  const uint64_t ain = (blk_len + n - 1) / n, aout = (nout + n - 1) / n;
  const uint64_t fit = std::min((uint64_t)(kWIn - 16) * 5u / (6u * ain + 10u),
                                (uint64_t)(kWOut - 16) * 5u / (6u * aout + 10u));
  if (fit >= (uint64_t)kWave && fit < tl) tl = fit;
  const uint64_t per_block = (((n + cus - 1) / cus + tl - 1) / tl) * tl;
  const unsigned grid = (unsigned)((n + per_block - 1) / per_block);
  RsArgs a{blk, blk_len, pos, limit, prefix, n, out, out_off, next, out_len, status, sc_start, sc_hend, sc_kind,
           fallback, gen, wg_agg};
  MHQ_DBG_SET_MEM(out, out + (blk_len / 5 * 8 + (blk_len % 5) * 8 / 5 + 1), blk, blk + ((blk_len + 15) & ~(uint64_t)15));
#ifdef MHQ_DBG_CRUMBS
  crumbs_arm(a, grid, per_block, tl, s);
#endif
  read_fused_kernel<<<dim3(grid), dim3(kT), 0, s>>>(a, t.lut1, t.lut2, t.len, per_block, (uint32_t)tl);
  return hipGetLastError();
}


// The fallback's grid and tile length are launch_decode's (its parse and
// scan phases work on the decode's workgroup ranges).
hipError_t launch_read_fallback(const DevTables &t, const uint8_t *blk, uint64_t blk_len, const uint64_t *pos,
                                const uint64_t *limit, const uint8_t *prefix, uint64_t n, uint8_t *out,
                                uint64_t out_cap, uint64_t *out_off, uint32_t *out_len, uint8_t *status,
                                uint64_t *next, uint64_t *sc_start, uint32_t *sc_hend, uint8_t *sc_kind,
                                uint64_t *fallback, uint64_t *wg_agg, uint64_t *wg_fin, uint64_t gen, hipStream_t s) {
  if (n == 0) return hipSuccess;
  const uint64_t cus = (uint64_t)dev::device_cus();
  const uint64_t slots = cus * kWaves;
  const uint64_t rounds = (n + slots * kTile - 1) / (slots * kTile);
  const uint64_t tl = std::max<uint64_t>(1, (n + slots * rounds - 1) / (slots * rounds));
  const uint64_t per_block = (((n + cus - 1) / cus + tl - 1) / tl) * tl;
  const unsigned grid = (unsigned)((n + per_block - 1) / per_block);
  if (grid > kReadFallbackMaxWgs) return hipErrorInvalidConfiguration;
  RsFallback f{RsArgs{blk, blk_len, pos, limit, prefix, n, out, out_off, next, out_len, status, sc_start, sc_hend,
                      sc_kind, fallback, gen, wg_agg},
               out_cap, wg_agg, wg_fin, lookback_help_polls()};
  MHQ_DBG_SET_MEM(out, out + out_cap, blk, blk + ((blk_len + 15) & ~(uint64_t)15));
  read_fallback_kernel<<<dim3(grid), dim3(kT), 0, s>>>(f, t.lut1, t.lut2, t.len, per_block, (uint32_t)tl);
  return hipGetLastError();
}

#ifdef MHQ_DBG_BOUNDS
MHQ_DBG_READER(mhq_dbg_bounds_read)
#endif

#ifdef MHQ_DBG_CRUMBS
extern "C" int mhq_dbg_crumbs_dump(const char *path) {
  FILE *f = fopen(path, "wb");
  if (!f) return -1;
  const uint64_t hdr[24] = {0x6d6871637275ull, g_crumb_lanes, (uint64_t)g_crumb_args.blk, g_crumb_args.blk_len,
                            (uint64_t)g_crumb_args.pos, (uint64_t)g_crumb_args.limit,
                            (uint64_t)g_crumb_args.prefix, g_crumb_args.n, (uint64_t)g_crumb_args.out,
                            (uint64_t)g_crumb_args.out_off, (uint64_t)g_crumb_args.next,
                            (uint64_t)g_crumb_args.out_len, (uint64_t)g_crumb_args.status,
                            (uint64_t)g_crumb_args.sc_start, (uint64_t)g_crumb_args.sc_hend,
                            (uint64_t)g_crumb_args.sc_kind, (uint64_t)g_crumb_args.fallback,
                            (uint64_t)g_crumb_args.wg_agg, g_crumb_args.gen, g_crumb_geom[0], g_crumb_geom[1],
                            g_crumb_geom[2], 0, 0};
  fwrite(hdr, sizeof(hdr), 1, f);
  if (g_crumb_host) fwrite(g_crumb_host, 16, g_crumb_lanes, f);
  fclose(f);
  return 0;
}
#endif

}  // namespace mhq
