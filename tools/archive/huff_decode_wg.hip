// huff_decode_wg.hip -- gfx950 batch decode of RFC 7541 Huffman literals,
// workgroup-cooperative tiles.
//
// Semantics are those of huff_decode.hip (hc/huffman.go:102-121 driven to EOF
// as Reader.ReadString does, hc/io.go:85-96; contract in SURVEY.md §8a and
// the CPU restatement oracle/huff_oracle.c).
//
// Structure: one workgroup per CU, kW waves.  Wave 0 stages; the other waves
// decode.  A tile is up to kTMax consecutive literals whose input and output
// fit one of kNBuf LDS buffers.  The stager loads the tile's offsets and input
// into the buffer with LDS-DMA loads (global_load_lds_dwordx4: no registers,
// no byte swap -- the decoders swap words as they read them), computes each
// literal's place in the buffer, zeroes the output staging, sorts the
// literals by encoded length (longest first) and publishes the tile.
// Decoders claim sub-tiles of 64 consecutive ranks from an LDS counter: lane l
// decodes one literal, and the 64 literals of a sub-tile have about the same
// length, so the lanes of a wave finish together without pairing literals.
// The decoder that finishes a tile's last sub-tile stores the tile's output
// (aligned 16-B stores) and lengths, and frees the buffer for the stager.
// The stager and the decoders synchronise through LDS words only (a
// workgroup's waves share the CU's LDS; no global-memory hand-off).
#include <hip/hip_runtime.h>

#include <algorithm>

#include "huff_common.h"
#include "huff_kernels.h"
#include "huff_table.h"

#ifndef MHQ_WG_WAVES  // waves per workgroup (wave 0 stages)
#define MHQ_WG_WAVES 16
#endif
#ifndef MHQ_WG_NBUF  // tile buffers
#define MHQ_WG_NBUF 2
#endif
#ifndef MHQ_WG_TMAX  // most literals per tile
#define MHQ_WG_TMAX 896
#endif
#ifndef MHQ_WG_IN_PER_LIT  // input slot bytes per literal of kTMax
#define MHQ_WG_IN_PER_LIT 24
#endif
#ifndef MHQ_WG_OUT_PER_LIT  // output slot bytes per literal of kTMax
#define MHQ_WG_OUT_PER_LIT 40
#endif

namespace mhq {
namespace {

using namespace dev;

constexpr int kW = MHQ_WG_WAVES;
constexpr int kT = kW * kWave;
constexpr int kNBuf = MHQ_WG_NBUF;
constexpr int kTMax = MHQ_WG_TMAX;
constexpr int kInB = kTMax * MHQ_WG_IN_PER_LIT;    // input slot bytes (from the tile's 16-B aligned start)
constexpr int kOutB = kTMax * MHQ_WG_OUT_PER_LIT;  // output slot bytes (from the tile's 16-B aligned start)
constexpr int kBuckets = 64;
static_assert(kInB % 16 == 0 && kOutB % 16 == 0, "slots are whole 16-B chunks");
static_assert(kInB < 65536 && kOutB < 65536, "a literal's place packs into 16-bit halves");
constexpr int kRecQ = (kTMax + 1 + kWave - 1) / kWave;  // offset entries per stager lane (entry q*64 + lane)

struct alignas(16) Tile {
  alignas(16) uint32_t in_w[kInB / 4 + 4];    // input bytes as loaded (words little-endian); +4 words look-ahead slack
  alignas(16) uint32_t out_w[kOutB / 4 + 4];  // output staging (global layout, zeroed); +4 words slack
  uint32_t rec[kTMax + 1];                    // per boundary: input byte index | output byte index << 16
  uint32_t len[kTMax];                        // out_len | status << 31
  uint16_t order[kTMax];                      // literals by descending encoded length
};

// Sub-tile claims carry the tile's generation (k + 1, 12 bits) above the
// count: a decoder that comes back for more after the tile was flushed and
// the buffer restaged sees another generation and takes nothing.
constexpr uint32_t kGenShift = 20;
__device__ __forceinline__ uint32_t gen_of(uint32_t k) { return (k + 1u) & 0xfffu; }

struct Ctl {  // one buffer's control words (LDS; workgroup-scope atomics)
  uint32_t ready;     // k + 1 once tile k is published here
  uint32_t freed;     // k + 1 once tile k's results have left (the buffer may be refilled)
  uint32_t next_sub;  // generation << kGenShift | sub-tiles claimed
  uint32_t done_sub;  // sub-tiles finished
  uint32_t nsub, cnt, end, idelta, odelta, pad;
  uint64_t s;   // the tile's first literal
  uint64_t oa;  // 16-B aligned global address of output slot byte 0
};

struct Smem {
  uint32_t lut1[kLut1Size];
  uint16_t lut2[kLut2Size];
  uint8_t clen[256];
  uint32_t hist[kBuckets];
  Ctl ctl[kNBuf];
  Tile t[kNBuf];
};

#ifdef MHQ_DIAG_WG  // diagnostic build: timeline (s_memrealtime, 100 MHz ticks)
// per workgroup: [0] start, [1] first publish, [2] stager end, [3] tiles,
// per tile k < 16: 4 + 8k + {0 stage start, 1 offsets landed, 2 published, 3 freed,
//   4 input DMA issued, 5 records + ranks done, 6 last sub-tile done, 7 flush stores issued};
// per decoder wave w (132 + 4w): {0 ticks waiting for a tile, 1 ticks decoding, 2 sub-tiles, 3 end}
constexpr int kDiagT = 4, kDiagD = 132;
constexpr int kDiagSlots = kDiagD + 4 * 16;
__device__ unsigned long long g_wgdiag[1024 * kDiagSlots];
#define WGD(slot, v)                                                              \
  do {                                                                            \
    if ((threadIdx.x & 63) == 0) g_wgdiag[blockIdx.x * kDiagSlots + (slot)] = (v); \
  } while (0)
#define WGD_ADD(slot, v)                                                           \
  do {                                                                             \
    if ((threadIdx.x & 63) == 0) g_wgdiag[blockIdx.x * kDiagSlots + (slot)] += (v); \
  } while (0)
#define NOW() wall_clock64()
#else
#define WGD(slot, v) \
  do {               \
  } while (0)
#define WGD_ADD(slot, v) \
  do {                   \
  } while (0)
#endif

typedef __attribute__((address_space(3))) void lds_void;
typedef __attribute__((address_space(1))) const void g_void;

__device__ __forceinline__ uint32_t ld_acq(const uint32_t *p) {
  return __hip_atomic_load(p, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_WORKGROUP);
}
__device__ __forceinline__ void st_rel(uint32_t *p, uint32_t v) {
  __hip_atomic_store(p, v, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_WORKGROUP);
}
// Spins (with s_sleep) until *p == v; every lane reads the same LDS word.
__device__ __forceinline__ void wait_eq(const uint32_t *p, uint32_t v) {
  while (ld_acq(p) != v) __builtin_amdgcn_s_sleep(1);
}
__device__ __forceinline__ uint32_t uni(uint32_t v) { return __builtin_amdgcn_readfirstlane(v); }

// A code of 13..30 bits, or the all-ones EOS prefix (c >= 30), at the top of
// the 32 stream bits `win`: its symbol and length, length 0 for the EOS prefix.
__device__ __forceinline__ uint32_t long_code(const uint16_t *lut2, uint32_t win, uint32_t &sym) {
  const uint32_t nw = ~win;
  const uint32_t c = nw ? (uint32_t)__builtin_clz(nw) : 32u;
  if (c >= (uint32_t)kEosOnes) return 0;
  const uint32_t e2 = lut2[(c << kLut2SubBits) | ((win << (c + 1)) >> (32 - kLut2SubBits))];
  sym = e2 & 0xffu;
  return e2 >> 8;
}

// Stream word k of a slot loaded as-is: bits 32k..32k+31, MSB first.
__device__ __forceinline__ uint32_t sw(const uint32_t *in_w, uint32_t k) { return __builtin_bswap32(in_w[k]); }

// A literal's stream bits in registers: `bb` holds bits [p, kb) MSB-aligned
// (zeros below); `w` is stream word kb/32, read ahead.
struct BitBuf {
  uint64_t bb;
  uint32_t p, kb, w;
  __device__ __forceinline__ void init(const uint32_t *in_w, uint32_t p0) {
    p = p0;
    const uint32_t k = p0 >> 5;
    bb = (((uint64_t)sw(in_w, k) << 32) | sw(in_w, k + 1)) << (p0 & 31u);
    kb = (k + 2u) * 32u;
    w = sw(in_w, k + 2u);
  }
  // Tops the buffer up to >= 33 valid bits when it holds <= 32 (branch free;
  // the look-ahead word is re-read either way).
  __device__ __forceinline__ void refill(const uint32_t *in_w) {
    const uint32_t nb = kb - p;
    const bool need = nb <= 32u;
    bb |= (uint64_t)(need ? w : 0u) << ((32u - nb) & 63u);
    kb += need ? 32u : 0u;
    w = sw(in_w, kb >> 5);
  }
  __device__ __forceinline__ uint32_t top32() const { return (uint32_t)(bb >> 32); }
  // Takes the bit count from an entry's low byte (the shift uses bits [5:0]).
  __device__ __forceinline__ void consume(uint32_t e) {
    bb <<= (e & 63u);
    p += e & 0xffu;
  }
};

// Output bytes in registers: `acc` holds the bytes from 4*ow up, `ab` bits of
// it are decided.  The low word is OR-ed into the zeroed staging every step
// (idempotent), so words shared with a neighbouring literal need no ordering.
struct OutAcc {
  uint64_t acc;
  uint32_t ow, ab;
  __device__ __forceinline__ void init(uint32_t optr) {
    acc = 0;
    ow = optr >> 2;
    ab = (optr & 3u) * 8u;
  }
  __device__ __forceinline__ void put(uint32_t syms, uint32_t nbits) {
    acc |= (uint64_t)syms << ab;
    ab += nbits;
  }
  __device__ __forceinline__ void flush(uint32_t *out_w) {
    atomicOr(&out_w[ow], (uint32_t)acc);
    acc >>= ab & 32u;  // a completed word leaves
    ow += ab >> 5;
    ab &= 31u;
  }
  __device__ __forceinline__ uint32_t optr() const { return ow * 4u + (ab >> 3); }
};

// One fast step at bit p of a literal ending at endbit (p + 24 <= endbit):
// two LUT1 probes (<= 12 bits each) with no end or room check.  A long code
// or the EOS prefix has entry 0, which consumes and emits nothing, so the
// second probe meets it again: one check per step resolves it through LUT2.
// The EOS prefix (INVALID when a 31st bit follows) and a long code running
// past the end both finish the literal: `lim` = -1 ends the fast loop and
// `bad` carries the status.
__device__ __forceinline__ void fast_step(const Smem &sm, const uint32_t *in_w, uint32_t *out_w, BitBuf &in,
                                          OutAcc &out, uint32_t endbit, int &lim, uint32_t &bad) {
  uint32_t e = sm.lut1[in.top32() >> (32 - kLut1Bits)];
  out.put(e >> 16, (e >> 8) & 0xffu);
  in.consume(e);
  e = sm.lut1[in.top32() >> (32 - kLut1Bits)];
  if (e == 0) {  // a long code or the EOS prefix (the first probe, if it met one, took nothing)
    in.refill(in_w);
    uint32_t sym = 0;
    const uint32_t L = long_code(sm.lut2, in.top32(), sym);
    const uint32_t left = endbit - in.p;
    if (L == 0 || L > left) {
      bad = L == 0 && left > (uint32_t)kEosOnes;  // a 31st bit exists: nil child (hc/huffman.go:111-113)
      lim = -1;
    } else {
      e = L | (8u << 8) | (sym << 16);
    }
  }
  out.put(e >> 16, (e >> 8) & 0xffu);
  in.consume(e);
  in.refill(in_w);
  out.flush(out_w);
}

// The last (< 24) bits of a literal whose output region is not truncating:
// single probes while >= 12 bits are left, then one checked probe, which
// decodes every code that still fits (three codes need >= 15 bits; a long
// code cannot fit).  No EOS prefix can be INVALID here (that needs > 30 bits).
// Returns out_len.
__device__ __forceinline__ uint32_t decode_end(const Smem &sm, const uint32_t *in_w, uint32_t *out_w, uint32_t p,
                                               uint32_t endbit, uint32_t optr, uint32_t ostart) {
  BitBuf in;
  in.init(in_w, p);
  OutAcc out;
  out.init(optr);
  bool more = true;
  while (more && in.p + 12u <= endbit) {
    uint32_t e = sm.lut1[in.top32() >> (32 - kLut1Bits)];
    if (e == 0) {
      uint32_t sym = 0;
      const uint32_t L = long_code(sm.lut2, in.top32(), sym);
      more = L != 0 && L <= endbit - in.p;
      e = more ? (L | (8u << 8) | (sym << 16)) : 0u;
    }
    out.put(e >> 16, (e >> 8) & 0xffu);
    in.consume(e);
    in.refill(in_w);
    out.flush(out_w);
  }
  if (more) {
    const uint32_t e = sm.lut1[in.top32() >> (32 - kLut1Bits)];
    const uint32_t left = endbit - in.p;
    const uint32_t len0 = sm.clen[(e >> 16) & 0xffu];
    const uint32_t c8 = e == 0 ? 0u : ((e & 0xffu) <= left ? (e >> 8) & 0xffu : (len0 <= left ? 8u : 0u));
    out.put(__builtin_amdgcn_ubfe(e >> 16, 0, c8), c8);
  }
  atomicOr(&out_w[out.ow], (uint32_t)out.acc);
  if (out.ab > 32u) atomicOr(&out_w[out.ow + 1], (uint32_t)(out.acc >> 32));
  return out.optr() - ostart;
}

// The general checked loop (literals with a truncating output region):
// decodes literal bits [p, endbit) into staging bytes [optr, oend) one probe
// at a time, with the reference's end-of-literal and buffer-full rules
// (hc/huffman.go:102-121).  Returns out_len | status << 31.
__device__ __noinline__ uint32_t decode_checked(const Smem &sm, const uint32_t *in_w, uint32_t *out_w, uint32_t p,
                                                uint32_t endbit, uint32_t optr, uint32_t oend) {
  BitBuf in;
  in.init(in_w, p);
  OutAcc out;
  out.init(optr);
  const uint32_t ostart = optr;
  uint32_t bad = 0;
  bool fin = false;
  while (!fin) {
    in.refill(in_w);
    const uint32_t win = in.top32();
    const uint32_t left = endbit - in.p;
    const uint32_t e = sm.lut1[win >> (32 - kLut1Bits)];
    uint32_t tot = e & 0xffu, ns8 = (e >> 8) & 0xffu, syms = e >> 16, len0 = sm.clen[(e >> 16) & 0xffu];
    if (e == 0) {
      const uint32_t L = long_code(sm.lut2, win, syms);
      len0 = tot = L ? L : 0xffffffffu;  // the EOS prefix never fits: the literal ends here
      ns8 = 8u;
      bad |= L == 0 && left > (uint32_t)kEosOnes;  // a 31st bit exists: nil child
    }
    uint32_t c8 = tot <= left ? ns8 : (len0 <= left ? 8u : 0u);
    const uint32_t room = oend - out.optr();  // Read() stops once p is full (hc/huffman.go:104)
    c8 = room >= 2u ? c8 : min(c8, room * 8u);
    const uint32_t cons = c8 == 16u ? tot : (c8 ? len0 : 0u);
    out.put(__builtin_amdgcn_ubfe(syms, 0, c8), c8);
    in.bb <<= cons & 63u;
    in.p += cons;
    fin = c8 == 0;
    out.flush(out_w);
  }
  const uint32_t oend_got = out.optr();
  bad = oend_got != oend ? bad : 0u;
  return (oend_got - ostart) | (bad << 31);
}

// One literal, one lane, straight from global memory (a literal larger than a
// slot).  Same decision rules as the staged loops.
__device__ __noinline__ void decode_literal_global(const uint8_t *src, uint64_t nbytes, uint8_t *dst, uint64_t cap,
                                                   const Smem &sm, uint32_t *out_len, uint8_t *status) {
  const uintptr_t a0 = (uintptr_t)src & ~(uintptr_t)3;
  const uint32_t *wb = (const uint32_t *)a0;
  const uint64_t bit0 = ((uintptr_t)src & 3u) * 8u;
  const uint64_t endbit = bit0 + nbytes * 8u;
  const uint64_t lastw = nbytes ? ((uintptr_t)(src + nbytes - 1) - a0) >> 2 : 0;
  uint64_t p = bit0, n = 0;
  uint8_t st = 0;
  while (n < cap && p < endbit) {
    const uint64_t rem = endbit - p;
    const uint64_t k = p >> 5;
    const uint32_t s = (uint32_t)p & 31u;
    const uint32_t w0 = __builtin_bswap32(wb[k < lastw ? k : lastw]);
    const uint32_t w1 = __builtin_bswap32(wb[k + 1 < lastw ? k + 1 : lastw]);
    const uint32_t win = s ? (w0 << s) | (w1 >> (32u - s)) : w0;
    const uint32_t e = sm.lut1[win >> (32 - kLut1Bits)];
    if (e == 0) {  // a long code or the EOS prefix
      const uint32_t nw = ~win;
      const uint32_t c = nw ? (uint32_t)__builtin_clz(nw) : 32u;
      if (c >= (uint32_t)kEosOnes) {
        st = rem > (uint64_t)kEosOnes;
        break;
      }
      uint32_t sym = 0;
      const uint32_t L = long_code(sm.lut2, win, sym);
      if (L == 0 || L > rem) break;
      dst[n++] = (uint8_t)sym;
      p += L;
      continue;
    }
    const uint32_t tot = e & 0xffu, s0 = (e >> 16) & 0xffu, len0 = sm.clen[s0];
    if (len0 > rem) break;
    dst[n++] = (uint8_t)s0;
    if (((e >> 8) & 0xffu) == 16u && tot <= rem && n < cap) {
      dst[n++] = (uint8_t)(e >> 24);
      p += tot;
    } else {
      p += len0;
    }
  }
  *out_len = (uint32_t)n;
  *status = st;
}

// ---- the stager ---------------------------------------------------------

__device__ __forceinline__ void dma_wait() { asm volatile("s_waitcnt vmcnt(0)" ::: "memory"); }

// Copies `chunks` 16-B chunks from the 16-B aligned global address g into LDS
// at `lds` (16-B aligned), 1 KiB per wave instruction (LDS-DMA).  Lanes past
// the last chunk stay inactive, so nothing past the run is written; the last
// chunk holds a wanted byte, so no load leaves the buffer (an aligned chunk
// never crosses a page).
__device__ __forceinline__ void dma_chunks(uint32_t *lds, const uint8_t *g, uint32_t chunks, uint32_t lane) {
  for (uint32_t c0 = 0; c0 < chunks; c0 += kWave) {
    if (c0 + lane < chunks)
      __builtin_amdgcn_global_load_lds((g_void *)(g + 16u * (c0 + lane)), (lds_void *)(lds + 4u * c0), 16, 0, 0);
  }
}

#ifdef MHQ_DIAG_WG
__device__ __shared__ uint32_t g_diag_k;
#endif

// The builtin returns int: each half goes through uint32_t, or a low word
// >= 2^31 would sign-extend over the high one (offsets of 2-4 GiB, 6-8 GiB...).
__device__ __forceinline__ uint64_t uniform64(uint64_t v) {
  return (uint64_t)(uint32_t)__builtin_amdgcn_readfirstlane((uint32_t)v) |
         ((uint64_t)(uint32_t)__builtin_amdgcn_readfirstlane((uint32_t)(v >> 32)) << 32);
}
// Lane l gets lane l+1's value (DPP wave_shl:1); lane 63 gets `last`.
__device__ __forceinline__ uint32_t from_next_lane(uint32_t v, uint32_t last) {
  return (uint32_t)__builtin_amdgcn_update_dpp((int)last, (int)v, 0x130, 0xf, 0xf, false);
}

// The stager keeps the next tile's offsets in registers: the low 32 bits of
// entry j = q*64 + lane of in_off / out_off from literal cur (entries past
// cur + want repeat the last one; a tile's spans are far below 2^32, so the
// low halves give exact differences), loaded a whole tile ahead, so planning
// a tile needs no LDS round trip (the decoders keep the LDS busy; every
// stager round trip waits behind their probes).
struct Stager {
  uint64_t cur;   // next literal to stage
  uint32_t want;  // literals whose offsets are in flight (cur .. cur + want)
  uint64_t ib, ob;  // in_off[cur], out_off[cur]
  uint32_t oi[kRecQ], oo[kRecQ];
  __device__ __forceinline__ void prefetch(const uint64_t *__restrict__ in_off, const uint64_t *__restrict__ out_off,
                                           uint64_t L1, uint32_t lane) {
    want = (uint32_t)min((uint64_t)kTMax, L1 > cur ? L1 - cur : 0);
    const uint64_t c = min(cur, L1);
    ib = in_off[c];
    ob = out_off[c];
    const uint32_t *lo_i = (const uint32_t *)(in_off + c), *lo_o = (const uint32_t *)(out_off + c);
#pragma unroll
    for (int q = 0; q < kRecQ; q++) {
      const uint32_t j = min((uint32_t)(q * kWave) + lane, want);
      oi[q] = __builtin_nontemporal_load(lo_i + 2u * j);  // little-endian: the low half
      oo[q] = __builtin_nontemporal_load(lo_o + 2u * j);
    }
  }
};

// Stages the literals from st.cur into buffer b (free), whose offsets are in
// st's registers; starts the next tile's offsets.  Returns the literals taken
// (0: literal st.cur alone is larger than a slot; it is not consumed).  The
// input DMA goes first; the records and the sort run while it is in flight.
__device__ uint32_t stage_tile(Smem &sm, int b, Stager &st, uint64_t L1, const uint8_t *__restrict__ in,
                               const uint64_t *__restrict__ in_off, uint64_t in_bias, uint8_t *__restrict__ out,
                               const uint64_t *__restrict__ out_off, uint64_t out_bias, uint32_t lane) {
  Tile &t = sm.t[b];
  Ctl &c = sm.ctl[b];
  const uint32_t want = st.want;
  const uint64_t ib = uniform64(st.ib), ob = uniform64(st.ob);
  const uint8_t *ia = in + (ib - in_bias);
  uint8_t *oa = out + (ob - out_bias);
  const uint32_t idelta = (uint32_t)((uintptr_t)ia & 15u), odelta = (uint32_t)((uintptr_t)oa & 15u);
  const uint32_t ib32 = (uint32_t)ib, ob32 = (uint32_t)ob;
#define RI(q) (st.oi[q] - ib32 + idelta)
#define RO(q) (st.oo[q] - ob32 + odelta)
  // the longest prefix [0, m) whose boundary m fits both slots: m + 1 is the
  // first boundary that does not (spans grow with j, so the first misfit
  // comes before the low halves could wrap)
  uint32_t m = want;
#pragma unroll
  for (int q = 0; q < kRecQ; q++) {
    const uint32_t j = (uint32_t)(q * kWave) + lane;
    const uint64_t bad = __ballot(j >= 1u && j <= want && (RI(q) > (uint32_t)kInB || RO(q) > (uint32_t)kOutB));
    if (bad && m == want) m = (uint32_t)(q * kWave) + (uint32_t)__builtin_ctzll(bad) - 1u;
  }
  if (m == 0) return 0;
  uint32_t in_bytes = 0, out_bytes = 0;
#pragma unroll
  for (int q = 0; q < kRecQ; q++) {
    if ((uint32_t)q == m / kWave) {
      in_bytes = __builtin_amdgcn_readlane(RI(q), m % kWave);
      out_bytes = __builtin_amdgcn_readlane(RO(q), m % kWave);
    }
  }
  // this tile's input (nothing for an all-empty tile, whose aligned chunk may lie past the buffer)
  if (in_bytes > idelta) dma_chunks(t.in_w, ia - idelta, (in_bytes + 15u) >> 4, lane);
#ifdef MHQ_DIAG_WG
  if (g_diag_k < 16) WGD(kDiagT + 8 * g_diag_k + 4, NOW());
#endif
  // records and length buckets
  sm.hist[lane] = 0;
  uint32_t rk[kRecQ];
#pragma unroll
  for (int q = 0; q < kRecQ; q++) {
    const uint32_t j = (uint32_t)(q * kWave) + lane;
    const uint32_t ri = RI(q);
    if (j <= m) t.rec[j] = ri | RO(q) << 16;
    const uint32_t nxt = from_next_lane(ri, __builtin_amdgcn_readlane(RI(q + 1 < kRecQ ? q + 1 : q), 0));
    const uint32_t bytes = (j < m ? nxt : ri) - ri;
    const uint32_t bk = bytes < 48u ? bytes : min(48u + ((bytes - 48u) >> 4), (uint32_t)kBuckets - 1u);
    rk[q] = (uint32_t)kBuckets - 1u - bk;
  }
#undef RI
#undef RO
  wave_sync();
#pragma unroll
  for (int q = 0; q < kRecQ; q++) {
    const uint32_t j = (uint32_t)(q * kWave) + lane;
    if (j < m) rk[q] |= atomicAdd(&sm.hist[rk[q]], 1u) << 8;
  }
  // the next tile's offsets (this tile's are no longer needed)
  st.cur += m;
  st.prefetch(in_off, out_off, L1, lane);
#ifdef MHQ_DIAG_WG
  if (g_diag_k < 16) WGD(kDiagT + 8 * g_diag_k + 5, NOW());
#endif
  // zero the output slot (16-B chunks, a few in flight per lane)
  {
    const uint32_t nq = ((out_bytes + 15u) >> 4) + 1u;
    for (uint32_t q = lane; q < nq; q += 4u * kWave) {
#pragma unroll
      for (int u = 0; u < 4; u++)
        if (q + (uint32_t)u * kWave < nq) *(u32x4 *)(t.out_w + 4u * (q + (uint32_t)u * kWave)) = u32x4{0u, 0u, 0u, 0u};
    }
  }
  wave_sync();
  {
    const uint32_t h = sm.hist[lane];
    sm.hist[lane] = wave_incl_scan(h) - h;
  }
  wave_sync();
#pragma unroll
  for (int q = 0; q < kRecQ; q++) {
    const uint32_t j = (uint32_t)(q * kWave) + lane;
    if (j < m) t.order[sm.hist[rk[q] & 0xffu] + (rk[q] >> 8)] = (uint16_t)j;
  }
  c.nsub = (m + kWave - 1u) / kWave;
  c.cnt = m;
  c.end = 0;
  c.idelta = idelta;
  c.odelta = odelta;
  c.s = st.cur - m;
  c.oa = (uint64_t)(uintptr_t)(oa - odelta);
  c.done_sub = 0;
  // the input has landed (only the next offsets, issued after it, may still be in flight)
  asm volatile("s_waitcnt vmcnt(%0)" ::"n"(2 * kRecQ + 2) : "memory");
  wave_sync();
  return m;
}

// ---- the decoders -------------------------------------------------------

__device__ __forceinline__ void decode_sub(const Smem &sm, Tile &t, uint32_t m, uint32_t j, uint32_t lane) {
  const uint32_t r = j * kWave + lane;
  const bool has = r < m;
  const uint32_t lit = has ? t.order[r] : t.order[0];
  const uint32_t r0 = t.rec[lit], r1 = t.rec[lit + 1];
  const uint32_t p = (r0 & 0xffffu) * 8u, endbit = (r1 & 0xffffu) * 8u;
  const uint32_t optr = r0 >> 16, oend = r1 >> 16;
  const bool roomy = oend - optr >= (endbit - p) / 5u;  // floor(bits/5) bytes: the most any input can produce
  if (!has) return;
  if (!roomy) {
    t.len[lit] = decode_checked(sm, t.in_w, t.out_w, p, endbit, optr, oend);
    return;
  }
  uint32_t q = p, o = optr, bad = 0;
  bool done = false;
  if (p + 24u <= endbit) {
    BitBuf in;
    in.init(t.in_w, p);
    OutAcc out;
    out.init(optr);
    int lim = (int)endbit - 24;
    while ((int)in.p <= lim) fast_step(sm, t.in_w, t.out_w, in, out, endbit, lim, bad);
    atomicOr(&t.out_w[out.ow], (uint32_t)out.acc);  // bits of a completed word not yet written
    q = in.p;
    o = out.optr();
    done = lim < 0;
  }
  t.len[lit] = done ? (o - optr) | (bad << 31) : decode_end(sm, t.in_w, t.out_w, q, endbit, o, optr);
}

// The last decoder of tile k: the tile's output region (up to the last
// literal's last decoded byte) and its lengths leave; the buffer is freed.
// Eight 16-B chunks per lane are read before any is stored, so one LDS
// round trip covers 8 KiB of output.
__device__ __forceinline__ void flush_tile(Smem &sm, int b, uint32_t k, uint32_t *__restrict__ out_len,
                                           uint8_t *__restrict__ status, uint32_t lane) {
  Tile &t = sm.t[b];
  Ctl &c = sm.ctl[b];
#ifdef MHQ_WG_PRIO
  __builtin_amdgcn_s_setprio(2);
#endif
#ifdef MHQ_DIAG_WG
  if (k < 16) WGD(kDiagT + 8 * k + 6, NOW());
#endif
  const uint32_t m = c.cnt, lo = c.odelta;
  const uint64_t s = c.s;
  const uint32_t hi = (t.rec[m - 1] >> 16) + (t.len[m - 1] & 0x7fffffffu);
  uint8_t *o_al = (uint8_t *)(uintptr_t)c.oa;
  const uint8_t *lds = (const uint8_t *)t.out_w;
  if (hi > lo) {
    const uint32_t f0 = (lo + 15u) >> 4, f1 = hi >> 4;  // whole chunks [f0, f1)
    constexpr int kU = 8;
    for (uint32_t c0 = f0; c0 < f1; c0 += kU * kWave) {
      u32x4 v[kU];
#pragma unroll
      for (int u = 0; u < kU; u++) {
        const uint32_t q = c0 + (uint32_t)u * kWave + lane;
        if (q < f1) v[u] = *(const u32x4 *)(lds + (q << 4));
      }
#pragma unroll
      for (int u = 0; u < kU; u++) {
        const uint32_t q = c0 + (uint32_t)u * kWave + lane;
        if (q < f1) __builtin_nontemporal_store(v[u], (u32x4 *)(o_al + (q << 4)));
      }
    }
    // the bytes of the (at most two) partial chunks at the ends
    const uint32_t head_end = min(hi, f0 << 4), tail_start = max(head_end, f1 << 4);
    const uint32_t x = lane < 16 ? lo + lane : tail_start + lane - 16u;
    if (lane < 32 && x < (lane < 16 ? head_end : hi)) o_al[x] = lds[x];
  }
  constexpr int kL = (kTMax + kWave - 1) / kWave;
  uint32_t v[kL];
#pragma unroll
  for (int q = 0; q < kL; q++) {
    const uint32_t j = (uint32_t)q * kWave + lane;
    v[q] = j < m ? t.len[j] : 0u;
  }
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");  // every LDS read of the buffer is back
  wave_sync();
#ifdef MHQ_DIAG_WG
  if (k < 16) WGD(kDiagT + 8 * k + 7, NOW());
#endif
  if (lane == 0) st_rel(&c.freed, k + 1u);
#pragma unroll
  for (int q = 0; q < kL; q++) {
    const uint32_t j = (uint32_t)q * kWave + lane;
    if (j < m) {
      out_len[s + j] = v[q] & 0x7fffffffu;
      status[s + j] = (uint8_t)(v[q] >> 31);
    }
  }
#ifdef MHQ_WG_PRIO
  __builtin_amdgcn_s_setprio(0);
#endif
}

__global__ __launch_bounds__(kT) void decode_wg_kernel(const uint8_t *__restrict__ in,
                                                       const uint64_t *__restrict__ in_off, uint64_t in_bias,
                                                       uint64_t n, uint8_t *__restrict__ out,
                                                       const uint64_t *__restrict__ out_off, uint64_t out_bias,
                                                       uint32_t *__restrict__ out_len, uint8_t *__restrict__ status,
                                                       const uint32_t *__restrict__ g_lut1,
                                                       const uint16_t *__restrict__ g_lut2,
                                                       const uint8_t *__restrict__ g_len, uint64_t per_block) {
  __shared__ Smem sm;
  const uint32_t tid = threadIdx.x;
  const uint32_t lane = tid % kWave;
  const uint32_t wave = tid / kWave;
  const uint64_t L0 = (uint64_t)blockIdx.x * per_block;
  if (L0 >= n) return;
  const uint64_t L1 = min(L0 + per_block, n);
  for (uint32_t i = tid; i < kLut1Size / 4; i += kT) ((u32x4 *)sm.lut1)[i] = ((const u32x4 *)g_lut1)[i];
  for (uint32_t i = tid; i < kLut2Size / 8; i += kT) ((u32x4 *)sm.lut2)[i] = ((const u32x4 *)g_lut2)[i];
  if (tid < 64) ((uint32_t *)sm.clen)[tid] = ((const uint32_t *)g_len)[tid];
  if (tid < (uint32_t)kNBuf) {
    sm.ctl[tid].ready = 0;
    sm.ctl[tid].freed = 0;
  }
  __syncthreads();

#ifdef MHQ_DIAG_WG
  if (tid == 0) {
    for (int q = 0; q < kDiagSlots; q++) g_wgdiag[blockIdx.x * kDiagSlots + q] = 0;
    g_wgdiag[blockIdx.x * kDiagSlots] = NOW();
  }
  __syncthreads();
#endif
  if (wave == 0) {  // the stager
#ifdef MHQ_WG_PRIO
    __builtin_amdgcn_s_setprio(3);  // wins instruction issue against the decoders of its SIMD
#endif
    Stager st;
    st.cur = L0;
    st.prefetch(in_off, out_off, L1, lane);
    for (uint32_t k = 0;; k++) {
      const int b = (int)(k % kNBuf);
#ifdef MHQ_DIAG_WG
      if (k >= (uint32_t)kNBuf && k - kNBuf < 16) {
        wait_eq(&sm.ctl[b].freed, k - kNBuf + 1u);
        WGD(kDiagT + 8 * (k - kNBuf) + 3, NOW());
      }
      if (lane == 0) g_diag_k = k;
      if (k < 16) WGD(kDiagT + 8 * k, NOW());
      WGD(3, k);
#endif
      if (k >= (uint32_t)kNBuf) wait_eq(&sm.ctl[b].freed, k - kNBuf + 1u);
      uint32_t m = 0;
      while (st.cur < L1) {
        m = stage_tile(sm, b, st, L1, in, in_off, in_bias, out, out_off, out_bias, lane);
        if (m) break;
        // literal st.cur alone does not fit a slot: one lane decodes it from global memory
        const uint64_t cur = st.cur;
        if (lane == 0) {
          const uint64_t ib = in_off[cur], ie = in_off[cur + 1], ob = out_off[cur], oe = out_off[cur + 1];
          decode_literal_global(in + (ib - in_bias), ie - ib, out + (ob - out_bias), oe - ob, sm, out_len + cur,
                                status + cur);
        }
        st.cur = cur + 1;
        st.prefetch(in_off, out_off, L1, lane);
      }
#ifdef MHQ_DIAG_WG
      if (k < 16) WGD(kDiagT + 8 * k + 1, NOW());
#endif
      if (m == 0) {  // no more literals
        dma_wait();
        sm.ctl[b].end = 1;
        sm.ctl[b].cnt = 0;
        sm.ctl[b].nsub = 0;
        wave_sync();
        if (lane == 0) st_rel(&sm.ctl[b].ready, k + 1u);
        WGD(2, NOW());
        return;
      }
#ifdef MHQ_DIAG_WG
      if (k < 16) WGD(kDiagT + 8 * k + 2, NOW());
      if (k == 0) WGD(1, NOW());
#endif
      if (lane == 0) {
        sm.ctl[b].next_sub = gen_of(k) << kGenShift;
        st_rel(&sm.ctl[b].ready, k + 1u);
      }
    }
  }

  // decoders
#ifdef MHQ_DIAG_WG
  unsigned long long t_wait = 0, t_work = 0, n_sub = 0;
#endif
  for (uint32_t k = 0;; k++) {
    const int b = (int)(k % kNBuf);
    Ctl &c = sm.ctl[b];
#ifdef MHQ_DIAG_WG
    const unsigned long long t0 = NOW();
    wait_eq(&c.ready, k + 1u);
    t_wait += NOW() - t0;
    if (uni(c.end)) {
      WGD(kDiagD + 4 * (wave - 1), t_wait);
      WGD(kDiagD + 4 * (wave - 1) + 1, t_work);
      WGD(kDiagD + 4 * (wave - 1) + 2, n_sub);
      WGD(kDiagD + 4 * (wave - 1) + 3, NOW());
      return;
    }
#else
    wait_eq(&c.ready, k + 1u);
    if (uni(c.end)) return;
#endif
    const uint32_t nsub = uni(c.nsub), m = uni(c.cnt);
    const uint32_t g = gen_of(k);
    for (;;) {
      uint32_t j = nsub;  // claim a sub-tile of this generation, if one is left
      if (lane == 0) {
        uint32_t v = ld_acq(&c.next_sub);
        while ((v >> kGenShift) == g && (v & ((1u << kGenShift) - 1u)) < nsub) {
          const uint32_t w = atomicCAS(&c.next_sub, v, v + 1u);
          if (w == v) {
            j = v & ((1u << kGenShift) - 1u);
            break;
          }
          v = w;
        }
      }
      j = uni(j);
      if (j >= nsub) break;
#ifdef MHQ_DIAG_WG
      const unsigned long long t1 = NOW();
#endif
      decode_sub(sm, sm.t[b], m, j, lane);
#ifdef MHQ_DIAG_WG
      t_work += NOW() - t1;
      n_sub++;
#endif
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");  // this wave's output and lengths are in the slot
      wave_sync();
      uint32_t d = 0;
      if (lane == 0) d = __hip_atomic_fetch_add(&c.done_sub, 1u, __ATOMIC_ACQ_REL, __HIP_MEMORY_SCOPE_WORKGROUP);
      d = uni(d);
      if (d == nsub - 1u) flush_tile(sm, b, k, out_len, status, lane);
    }
  }
}

}  // namespace

#ifdef MHQ_DIAG_WG
extern "C" int mhq_diag_wg(unsigned long long *out, int n) {
  const int m = n < 1024 * kDiagSlots ? n : 1024 * kDiagSlots;
  return hipMemcpyFromSymbol(out, HIP_SYMBOL(g_wgdiag), m * sizeof(unsigned long long)) == hipSuccess ? kDiagSlots
                                                                                                       : -1;
}
#endif

hipError_t launch_decode_wg(const DevTables &t, const uint8_t *in, const uint64_t *in_off, uint64_t in_bias,
                            uint64_t n, uint8_t *out, const uint64_t *out_off, uint64_t out_bias, uint32_t *out_len,
                            uint8_t *status, hipStream_t s) {
  if (n == 0) return hipSuccess;
  const uint64_t cus = (uint64_t)dev::device_cus();
  const uint64_t per_block = std::max<uint64_t>(1, (n + cus - 1) / cus);
  const unsigned grid = (unsigned)((n + per_block - 1) / per_block);
  decode_wg_kernel<<<dim3(grid), dim3(kT), 0, s>>>(in, in_off, in_bias, n, out, out_off, out_bias, out_len, status,
                                                   t.lut1, t.lut2, t.len, per_block);
  return hipGetLastError();
}

}  // namespace mhq
