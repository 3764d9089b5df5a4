// huff_decode_dev.h -- device core of the gfx950 batch decode, shared by the
// decode kernel (huff_decode.hip) and the fused read_strings kernels
// (read_strings.hip).  The design is described in huff_decode.hip.
#pragma once
#include <hip/hip_runtime.h>
#include <algorithm>
#include "huff_common.h"
#include "huff_kernels.h"
#include "huff_table.h"

#ifndef MHQ_DEC_WAVES  // waves per workgroup (one workgroup per CU)
#define MHQ_DEC_WAVES 12
#endif
#ifndef MHQ_DEC_TILE  // most literals per wave tile (64 < tile <= 128)
#define MHQ_DEC_TILE 128
#endif
#ifndef MHQ_DEC_PF  // 16-B input chunks per lane staged from registers: a wave's input slice is 1 KiB * PF
#define MHQ_DEC_PF 4
#endif
#ifndef MHQ_DEC_STEPS  // masked steps per end test of the probe loop (the plain decode)
#define MHQ_DEC_STEPS 3
#endif
#ifndef MHQ_DEC_PAIR  // 1: a group's steps in pairs on one window read (win_pair)
#define MHQ_DEC_PAIR 1
#endif
#ifndef MHQ_DEC_STEPS_GAPS  // the same for the in_end decode of framed strings (read_strings; 3 since r05j: -1..-4 %)
#define MHQ_DEC_STEPS_GAPS 3
#endif
// The plain decode's out-of-line helper (the checked loop) is a called
// function; its streamed long literals are inlined at the compiler's choice.
// The in_end decode (kGaps: read_strings, decode_kernel<true>) inlines both:
// a call there spilled what was live across it (read_fused_kernel: 11 VGPRs
// and 74 SGPRs, 48 B of scratch a lane) and reached LDS through generic
// (flat) pointers; inlined, the read kernels have no call, no flat access
// and no scratch.
#define MHQ_CALLEE __noinline__
#define MHQ_CALLEE_LONG
#ifndef MHQ_DEC_WOUT  // a wave's output slice (bytes, multiple of 16)
#define MHQ_DEC_WOUT 6448
#endif

namespace mhq {
namespace {

using namespace dev;

constexpr int kWaves = MHQ_DEC_WAVES;
constexpr int kT = kWaves * kWave;
constexpr int kTile = MHQ_DEC_TILE;  // most literals per wave tile
static_assert(kTile > kWave && kTile <= 2 * kWave, "a lane decodes one or two literals of a tile");
constexpr int kPF = MHQ_DEC_PF;
constexpr int kWIn = kPF * kWave * 16;  // input slice bytes (from the tile's 16-B aligned start)
constexpr int kWOut = MHQ_DEC_WOUT;     // output slice bytes (from the tile's 16-B aligned start)
constexpr int kBuckets = 64;
constexpr int kOutRounds = (kWOut + 16 * kWave - 1) / (16 * kWave);  // store_out_batched rounds of a slice
// wave priority while a wave stages, flushes and sorts a tile (its serial
// phases), so they do not wait behind the other waves' probe loops (north
// star 42.8 -> 41.8-42.0 us, round 2)
constexpr int kPhasePrio = 3;
static_assert(kWOut % 16 == 0, "output slice must be whole 16-B chunks");

// (16-B aligned: its 16-B LDS accesses are single ds_*_b128, not split pairs)
struct alignas(16) WaveSmem {
  uint32_t in_w[kWIn / 4 + 4];    // stream words, byte-swapped; +4 words of look-ahead slack
  uint32_t out_w[kWOut / 4 + 4];  // output staging (global layout, zero-filled); +4 words slack
  uint32_t rec[kTile + 1];        // per boundary: input byte index | output byte index << 16
  uint32_t len[kTile];            // out_len | status << 31, by literal
  uint32_t hist[kBuckets];
  uint8_t order[kTile];  // literals by descending encoded length
};

struct Smem {
  uint32_t lut1[kLut1Size];
  uint16_t lut2[kLut2Size];
  uint8_t clen[256];  // code length per symbol (len0 of a LUT1 entry, for the checked loop)
  uint32_t next_tile;
  uint32_t tl;  // the tile length this launch uses (see decode_kernel)
  WaveSmem w[kWaves];
};

#ifdef MHQ_DBG_BOUNDS
// Diagnostic build (-DMHQ_DBG_BOUNDS): the bounds of the LDS records, the
// fast loop's output word and the global stores of the decode and read path
// are checked where they are formed; a violation is recorded -- a code and two
// values, the first 16 -- never faulted on.  mhq_dbg_bounds_decode /
// mhq_dbg_bounds_read (one per translation unit) read and clear the records.
__device__ unsigned long long g_dbg[1 + 3 * 16];
__device__ __noinline__ void dbg_fail(uint32_t code, uint64_t a, uint64_t b) {
  const unsigned long long k = atomicAdd(&g_dbg[0], 1ull);
  if (k < 16) {
    g_dbg[1 + 3 * k] = code;
    g_dbg[2 + 3 * k] = a;
    g_dbg[3 + 3 * k] = b;
  }
}
#define DBG_CHECK(c, code, a, b)                                         \
  do {                                                                   \
    if (!(c)) dbg_fail((code), (uint64_t)(a), (uint64_t)(b));            \
  } while (0)
// Guards (the same build): an access whose address fails its check is
// recorded and SKIPPED, so a bad address shows up as a record instead of a
// fault.  g_dbg_mem: the global byte ranges the read path may write (the
// output) and read (the block), set by the read launchers (0: unchecked).
__device__ uint64_t g_dbg_mem[4];
__device__ __forceinline__ bool dbg_out_ok(const void *p, uint64_t bytes) {
  const uint64_t a = (uint64_t)(uintptr_t)p;
  return g_dbg_mem[1] == 0 || (a >= g_dbg_mem[0] && a + bytes <= g_dbg_mem[1]);
}
__device__ __forceinline__ bool dbg_in_ok(const void *p, uint64_t bytes) {
  const uint64_t a = (uint64_t)(uintptr_t)p;
  return g_dbg_mem[3] == 0 || (a >= g_dbg_mem[2] && a + bytes <= g_dbg_mem[3]);
}
// an LDS address (generic or local) inside the decode's allocation
__device__ __forceinline__ bool dbg_lds_ok(const void *p, uint64_t bytes) {
  return (uint32_t)(uintptr_t)p + bytes <= 163840u;
}
#define DBG_OK(c, code, a, b) ((c) || (dbg_fail((code), (uint64_t)(a), (uint64_t)(b)), false))
#define MHQ_DBG_SET_MEM(out_lo, out_hi, in_lo, in_hi)                                          \
  do {                                                                                       \
    const uint64_t _m[4] = {(uint64_t)(out_lo), (uint64_t)(out_hi), (uint64_t)(in_lo), (uint64_t)(in_hi)}; \
    (void)hipMemcpyToSymbol(HIP_SYMBOL(g_dbg_mem), _m, sizeof(_m));                          \
  } while (0)
#define MHQ_DBG_READER(name)                                                                  \
  extern "C" int name(unsigned long long *out, int n) {                                       \
    unsigned long long h[1 + 3 * 16];                                                         \
    if (hipMemcpyFromSymbol(h, HIP_SYMBOL(g_dbg), sizeof(h)) != hipSuccess) return -1;        \
    for (int i = 0; i < n && i < 1 + 3 * 16; i++) out[i] = h[i];                              \
    unsigned long long z[1 + 3 * 16] = {0};                                                   \
    return hipMemcpyToSymbol(HIP_SYMBOL(g_dbg), z, sizeof(z)) == hipSuccess ? 0 : -1;         \
  }
#else
#define DBG_CHECK(c, code, a, b) \
  do {                           \
  } while (0)
#define DBG_OK(c, code, a, b) true
#define MHQ_DBG_SET_MEM(out_lo, out_hi, in_lo, in_hi) \
  do {                                                \
  } while (0)
#endif

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

// One literal, one lane, straight from global memory: literals too large for
// the staging slices.  Same decision rules as the staged loop.
template <class SM>
__device__ void decode_literal_global(const uint8_t *src, uint64_t nbytes, uint8_t *dst, uint64_t cap,
                                      const SM &sm, uint32_t *out_len, uint8_t *status) {
  const uint8_t *a8 = src - ((uintptr_t)src & 3u);
  const uintptr_t a0 = (uintptr_t)a8;
  const uint32_t *wb = (const uint32_t *)a8;
  const uint64_t bit0 = ((uintptr_t)src & 3u) * 8u;
  const uint64_t endbit = bit0 + nbytes * 8u;
  const uint64_t lastw = nbytes ? ((uintptr_t)(src + nbytes - 1) - a0) >> 2 : 0;
  uint64_t p = bit0, n = 0;
  uint8_t st = 0;
  while (n < cap && p < endbit) {
    const uint64_t rem = endbit - p;
    const uint64_t k = p >> 5;
    const uint32_t s = (uint32_t)p & 31u;
    const uint32_t *r0 = wb + (k < lastw ? k : lastw), *r1 = wb + (k + 1 < lastw ? k + 1 : lastw);
    CRUMB(50, r1);
    const uint32_t w0 = DBG_OK(dbg_in_ok(r0, 4), 20, r0, src) ? __builtin_bswap32(*r0) : 0u;
    const uint32_t w1 = DBG_OK(dbg_in_ok(r1, 4), 20, r1, src) ? __builtin_bswap32(*r1) : 0u;
    const uint32_t win = s ? (w0 << s) | (w1 >> (32u - s)) : w0;
    const uint32_t e = sm.lut1[win >> (32 - kLut1Bits)];
    CRUMB(51, dst + n);
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
      if (DBG_OK(dbg_out_ok(dst + n, 1), 21, dst + n, cap)) dst[n] = (uint8_t)sym;
      n++;
      p += L;
      continue;
    }
    const uint32_t tot = e & 0xffu, s0 = (e >> 16) & 0xffu, len0 = sm.clen[s0];
    if (len0 > rem) break;
    if (DBG_OK(dbg_out_ok(dst + n, 1), 21, dst + n, cap)) dst[n] = (uint8_t)s0;
    n++;
    if (((e >> 8) & 0xffu) == 16u && tot <= rem && n < cap) {
      if (DBG_OK(dbg_out_ok(dst + n, 1), 21, dst + n, cap)) dst[n] = (uint8_t)(e >> 24);
      n++;
      p += tot;
    } else {
      p += len0;
    }
  }
  *out_len = (uint32_t)n;
  *status = st;
}

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

// A literal's stream bits in registers: `bb` holds bits [p, kb) MSB-aligned
// (zeros below); `w` is staged word kb/32, read ahead.
struct BitBuf {
  uint64_t bb;
  uint32_t p, kb, w;
  const uint32_t *in_w;

  __device__ __forceinline__ void init(const uint32_t *words, uint32_t p0) {
    in_w = words;
    p = p0;
    const uint32_t k = p0 >> 5;
    bb = (((uint64_t)in_w[k] << 32) | in_w[k + 1]) << (p0 & 31u);
    kb = (k + 2u) * 32u;
    w = in_w[k + 2u];
  }
  // Tops the buffer up to >= 33 valid bits when it holds <= 32 (branch free;
  // the look-ahead word is re-read either way).
  __device__ __forceinline__ void refill() {
    const uint32_t nb = kb - p;
    const bool need = nb <= 32u;
    bb |= (uint64_t)(need ? w : 0u) << ((32u - nb) & 63u);
    kb += need ? 32u : 0u;
    w = in_w[kb >> 5];
  }
  __device__ __forceinline__ uint32_t top32() const { return (uint32_t)(bb >> 32); }
  // Takes the bit count from an entry's low byte (the shift uses bits [5:0]).
  __device__ __forceinline__ void consume(uint32_t e) {
    bb <<= (e & 63u);
    p += e & 0xffu;
  }
};

// The fast loop's output state: the output word is held as an LDS pointer
// (its address needs no arithmetic per step), and a step's output word is
// OR-ed whether or not a code crossed the literal's end -- a crossing makes
// the whole piece be decoded again by the checked loop over a re-zeroed
// output region (decode_piece), so stray bits of a malformed literal never
// survive.
struct OutAccL {
  uint64_t acc;
  uint32_t ab;
  uint32_t *op;  // the word being filled
  __device__ __forceinline__ void init(uint32_t *out_w, uint32_t optr) {
    acc = 0;
    op = out_w + (optr >> 2);
    ab = (optr & 3u) * 8u;
  }
  __device__ __forceinline__ void put(uint32_t syms, uint32_t nbits) {
    acc |= (uint64_t)syms << ab;
    ab += nbits;
  }
  __device__ __forceinline__ uint32_t optr(const uint32_t *out_w) const {
    return (uint32_t)(op - out_w) * 4u + (ab >> 3);
  }
};
struct PendL {
  uint32_t *p, v;
};

// A literal's stream with no refill state: each step reads the two staged
// words holding its bit position (one ds_read2) and forms the window's top 32
// bits with one v_alignbit (no 64-bit shift, no word swap); bits past the
// literal's end are forced to ones (`msk`), so that a well-formed literal
// (at most 7 padding ones) meets >= 30 ones -- the EOS prefix -- at its
// padding and stops there, and a literal whose tail is not all ones decodes a
// code across its end, which `left < 0` shows (the piece is redone by the
// checked loop).  The state is the bit
// address minus one, so the words are those holding bits p-1 and p+31 and the
// shift ~pm & 31 is 31 - ((p-1) & 31): 0 when p is word-aligned (the second
// word whole), the first word's low bits otherwise.  Both probes and the stop
// test read these 32 bits (a first code takes at most 12, the second probe
// 12 more; a long code at most 30).
struct WinBuf3 {
  uint32_t pm;   // LDS bit address of the next bit, minus 1
  int32_t left;  // endbit - p
  uint32_t msk;  // ones from bit `left` on (MSB first): set with left, off the next step's read
  __device__ __forceinline__ void set_mask() { msk = (uint32_t)(0xffffffffull >> (uint32_t)min(max(left, 0), 32)); }
  __device__ __forceinline__ void init(const uint32_t *words, uint32_t p0, uint32_t endbit) {
    pm = 8u * (uint32_t)(uintptr_t)words + p0 - 1u;
    left = (int32_t)(endbit - p0);
    set_mask();
  }
  __device__ __forceinline__ uint32_t top() const {
    typedef __attribute__((address_space(3))) const uint32_t lds_u32;
    lds_u32 *w = (lds_u32 *)(uintptr_t)((pm >> 3) & ~3u);
    return __builtin_amdgcn_alignbit(w[0], w[1], ~pm) | msk;
  }
};

// One step on a window's 32 bits S (win_step32: S read from LDS at the step;
// win_pair: from three words read for two steps).
// kSafe (the streamed decode, huff_decode_stream.hip): a step that leaves
// `left` < 0 -- a code decoded across the literal's end -- pends nothing, so
// no byte of a malformed tail is ever OR-ed into the output (the literal is
// then decoded again by the exact path; the stream has no piece to redo).
template <bool kLong, bool kSafe = false>
__device__ __forceinline__ bool win_step_s(const Smem &sm, WinBuf3 &in, uint32_t S, OutAccL &out, PendL &pend,
                                           bool &stop) {
  stop = S >= 0xfffffffcu;
  uint32_t e = sm.lut1[S >> (32 - kLut1Bits)];
  atomicOr(pend.p, pend.v);
  bool lng = false;
  if (kLong && ((e == 0u) & !stop)) {  // a code of 13..29 bits (one branch: no short circuit)
    uint32_t sym = 0;
    const uint32_t L = long_code(sm.lut2, S, sym);
    e = L | (8u << 8) | (sym << 16);
    lng = true;
  }
  out.put(e >> 16, (e >> 8) & 0xffu);
  uint32_t e2 = sm.lut1[(S << (e & 31u)) >> (32 - kLut1Bits)];
  e2 = lng ? 0u : e2;
  out.put(e2 >> 16, (e2 >> 8) & 0xffu);
  const uint32_t n = (e & 0xffu) + (e2 & 0xffu);
  in.pm += n;
  in.left -= (int32_t)n;
  in.set_mask();
  pend.p = out.op;
  pend.v = (uint32_t)out.acc;
  if (kSafe) pend.v = in.left < 0 ? 0u : pend.v;
  const uint32_t t = out.ab & 32u;
  out.acc >>= t;
  out.op += t >> 5;
  out.ab &= 31u;
  return stop || in.left < 0;
}

template <bool kLong = true, bool kSafe = false>
__device__ __forceinline__ bool win_step32(const Smem &sm, WinBuf3 &in, OutAccL &out, PendL &pend, bool &stop) {
  return win_step_s<kLong, kSafe>(sm, in, in.top(), out, pend, stop);
}

// Two steps from one window read: three words from the first step's bit
// position cover the second step's too (a step without LUT2 moves at most
// 24 bits), so the second step's window comes from registers (one LDS round
// trip less on the step chain).  The words past a literal are the slice's
// look-ahead slack.
template <bool kLongB, bool kSafe = false>
__device__ __forceinline__ bool win_pair(const Smem &sm, WinBuf3 &in, OutAccL &out, PendL &pend, bool &stop) {
  typedef __attribute__((address_space(3))) const uint32_t lds_u32;
  lds_u32 *w = (lds_u32 *)(uintptr_t)((in.pm >> 3) & ~3u);
  const uint32_t k0 = in.pm >> 5, w0 = w[0], w1 = w[1], w2 = w[2];
  win_step_s<false, kSafe>(sm, in, __builtin_amdgcn_alignbit(w0, w1, ~in.pm) | in.msk, out, pend, stop);
  const bool hi = (in.pm >> 5) != k0;
  return win_step_s<kLongB, kSafe>(sm, in, __builtin_amdgcn_alignbit(hi ? w1 : w0, hi ? w2 : w1, ~in.pm) | in.msk, out,
                                   pend, stop);
}


// BitBuf over a long-path window (LDS-DMA): words left in memory byte order
// (each is byte-swapped as it is read), and the window's 16-B chunks stored
// XOR-swizzled: chunk c of lane l's window sits in slot c ^ (l % 8), so word k
// is at k ^ swz with swz = 4 (l % 8).  Lanes walking same-shaped literals read
// the same k together; unswizzled, all 32 lanes of a half-wave would hit one
// bank (windows are 32 words apart), swizzled they spread over 8 slots.
struct BitBufS {
  uint64_t bb;
  uint32_t p, kb, w, swz;
  const uint32_t *in_w;
  __device__ __forceinline__ uint32_t rd(const uint32_t *q, uint32_t k) const {
    return DBG_OK(dbg_lds_ok(q + (k ^ swz), 4), 28, (uintptr_t)(q + (k ^ swz)), k) ? __builtin_bswap32(q[k ^ swz]) : 0u;
  }
  __device__ __forceinline__ void init(const uint32_t *words, uint32_t p0, uint32_t swz_) {
    swz = swz_;
    in_w = words;
    p = p0;
    const uint32_t k = p0 >> 5;
    bb = (((uint64_t)rd(in_w, k) << 32) | rd(in_w, k + 1)) << (p0 & 31u);
    kb = (k + 2u) * 32u;
    w = rd(in_w, k + 2u);
  }
  __device__ __forceinline__ void refill() {
    const uint32_t nb = kb - p;
    const bool need = nb <= 32u;
    bb |= (uint64_t)(need ? w : 0u) << ((32u - nb) & 63u);
    kb += need ? 32u : 0u;
    w = rd(in_w, kb >> 5);
  }
  __device__ __forceinline__ uint32_t top32() const { return (uint32_t)(bb >> 32); }
  __device__ __forceinline__ void consume(uint32_t e) {
    bb <<= (e & 63u);
    p += e & 0xffu;
  }
};

// The general checked loop (literals with a truncating output region):
// decodes literal bits [p, endbit) into staging bytes [optr, oend) one probe
// at a time, with the reference's end-of-literal and buffer-full rules
// (hc/huffman.go:102-121).  Returns out_len | status << 31.
__device__ __forceinline__ uint32_t decode_checked_body(const Smem &sm, WaveSmem &ws, uint32_t p, uint32_t endbit,
                                                       uint32_t optr, uint32_t oend) {
  BitBuf in;
  in.init(ws.in_w, p);
  OutAcc out;
  out.init(optr);
  const uint32_t ostart = optr;
  uint32_t bad = 0;
  bool fin = false;
  while (!fin) {
    in.refill();
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
    DBG_CHECK(out.ow < (uint32_t)kWOut / 4u + 4u, 5, out.ow, oend);
    if (!DBG_OK(dbg_lds_ok(ws.out_w + out.ow, 4) && dbg_lds_ok(ws.in_w + (in.kb >> 5), 4), 22, out.ow, in.kb)) break;
    out.flush(ws.out_w);
  }
  const uint32_t oend_got = out.optr();
  bad = oend_got != oend ? bad : 0u;
  return (oend_got - ostart) | (bad << 31);
}
__device__ MHQ_CALLEE uint32_t decode_checked(const Smem &sm, WaveSmem &ws, uint32_t p, uint32_t endbit,
                                                uint32_t optr, uint32_t oend) {
  return decode_checked_body(sm, ws, p, endbit, optr, oend);
}
// (kGaps: inlined; see MHQ_CALLEE)
template <bool kGaps>
__device__ __forceinline__ uint32_t decode_checked_k(const Smem &sm, WaveSmem &ws, uint32_t p, uint32_t endbit,
                                                     uint32_t optr, uint32_t oend) {
  if constexpr (kGaps)
    return decode_checked_body(sm, ws, p, endbit, optr, oend);
  else
    return decode_checked(sm, ws, p, endbit, optr, oend);
}

// A literal's place in the staged tile.
// (kGaps: literal l's input ends at ws.len[l], not where literal l + 1
// starts; see decode_kernel.)
template <bool kGaps>
struct LitRef {
  uint32_t lit, p, endbit, optr, oend;
  __device__ __forceinline__ void load(const WaveSmem &ws, uint32_t l) {
    lit = l;
    const uint32_t r0 = ws.rec[l], r1 = ws.rec[l + 1];
    p = (r0 & 0xffffu) * 8u;
    endbit = (kGaps ? ws.len[l] : (r1 & 0xffffu)) * 8u;
    optr = r0 >> 16;
    oend = r1 >> 16;
  }
  // The output region holds floor(bits/5) bytes, the most any input can
  // produce: no room check is needed.
  __device__ __forceinline__ bool roomy() const { return oend - optr >= (endbit - p) / 5u; }
  // The most this literal can produce stays inside the output slice (its
  // last word included): run past a short region, it can only spoil bytes
  // that a redo of the piece re-zeroes, or the slice's unused tail.
  __device__ __forceinline__ bool in_slice() const { return optr + (endbit - p) / 5u + 4u <= (uint32_t)kWOut + 16u; }
};

#ifdef MHQ_DIAG_TIMELINE  // diagnostic build: per-wave timeline (s_memrealtime, 100 MHz)
constexpr int kTlSlots = 64;  // per wave: [0] start, [63] end, [56..58] opening, tile j < 11: 1 + 5j + {0 loads issued, 1 flushed, 2 sorted, 3 loop done, 4 decoded}
__device__ unsigned long long g_tl[1024 * 16 * kTlSlots];
#define TL(slot)                                                                                          \
  do {                                                                                                    \
    const int _s = (slot);                                                                                \
    if (threadIdx.x % kWave == 0 && _s < kTlSlots && _s >= 0)                                             \
      g_tl[(blockIdx.x * 16 + threadIdx.x / kWave) * kTlSlots + _s] = wall_clock64();                     \
  } while (0)
#else
#define TL(slot) \
  do {           \
  } while (0)
#endif
// Per-tile stamps of tile j < 11 (slots 1..55; 56..58 hold the opening's
// stamps, 63 the end); later tiles are not stamped (-1).
__device__ __forceinline__ int tl_slot(uint32_t j, int k) { return j < 11u ? k + 5 * (int)j : -1; }

// ---- per-wave tiles ------------------------------------------------------
// Workgroup b owns literals [L0, L1) = [b*R, (b+1)*R); tile t of it is
// literals L0 + 128t + [0, 128).  Wave w starts with tiles w and w + kWaves,
// then takes tiles from the LDS counter.
//
// Pipeline, per wave: while tile k decodes, tile k+1's input bytes and tile
// k+2's offsets are in flight in registers.  gfx9 counts stores in vmcnt
// too (in issue order with loads), so tile k-1's output and lengths are
// stored after tile k+1's loads are issued and before tile k decodes, and the
// decode issues no global memory operation: when tile k+1 starts, everything
// it waits for was issued a whole decode earlier.

typedef __attribute__((address_space(3))) void lds_void;
typedef __attribute__((address_space(1))) const void g_void;

struct TileOff {  // raw loads: in_off / out_off of literals s + 2*lane + {0, 1}, and of s + tile
  uint64_t i0, o0, ie, oe;
  uint32_t i1, o1;  // only their low words are used (tile-relative offsets): 32-bit loads
  uint32_t e0, e1;  // kGaps: in_end of the two literals (low words: in_end is a u32 array of them)
};
// The low word of a u64 offset.
__device__ __forceinline__ uint32_t lo32(const uint64_t *a, uint64_t j) { return ((const uint32_t *)a)[2u * j]; }

__device__ __forceinline__ uint32_t vzero() {
  uint32_t z;
  asm volatile("v_mov_b32 %0, 0" : "=v"(z));
  return z;
}

// The builtin returns int: each half goes through uint32_t, or a low word
// >= 2^31 would sign-extend over the high one (offsets of 2-4 GiB, 6-8 GiB...).
__device__ __forceinline__ uint64_t uniform64(uint64_t v) {
  return (uint64_t)(uint32_t)__builtin_amdgcn_readfirstlane((uint32_t)v) |
         ((uint64_t)(uint32_t)__builtin_amdgcn_readfirstlane((uint32_t)(v >> 32)) << 32);
}

// Offsets of the tile that starts at literal s (indices clamped to L1, so a
// tile past the range loads the range end).
// Indices relative to the tile's clamped start (a uniform base: the loads
// take a scalar base and a 32-bit lane offset, no 64-bit index arithmetic per
// lane); every workgroup range is under 2^32 literals.
struct TileIdx {
  uint64_t base;    // min(s, L1)
  uint32_t a0, a1;  // literals s + 2 lane + {0, 1}, clamped to L1
  uint32_t ae;      // literal s + tile, clamped to L1 (a vector index: see vzero)
  __device__ __forceinline__ TileIdx(uint64_t s, uint64_t L1, uint32_t tl, uint32_t lane) {
    base = min(s, L1);
    const uint32_t lim = (uint32_t)(L1 - base);
    a0 = min(2u * lane, lim);
    a1 = min(2u * lane + 1u, lim);
    ae = min(tl, lim) + vzero();  // keeps the uniform load a per-lane vector load
  }
};
// (in_end has n entries: indices clamped below L1, i.e. in_end[min(s + j, L1 - 1)])
template <bool kGaps>
__device__ __forceinline__ void load_end(TileOff &t, const uint32_t *__restrict__ in_end, uint64_t s, uint64_t L1,
                                         uint32_t lane) {
  if (!kGaps) return;
  const uint64_t eb = min(s, L1 - 1u);
  const uint32_t elim = (uint32_t)(L1 - 1u - eb);
  const uint32_t *e = in_end + eb;
  t.e0 = e[min(2u * lane, elim)];
  t.e1 = e[min(2u * lane + 1u, elim)];
}

template <bool kGaps>
__device__ __forceinline__ void load_off(TileOff &t, const uint64_t *__restrict__ in_off,
                                         const uint32_t *__restrict__ in_end, const uint64_t *__restrict__ out_off,
                                         uint64_t s, uint64_t L1, uint32_t tl, uint32_t lane) {
  const TileIdx x(s, L1, tl, lane);
  const uint64_t *ib = in_off + x.base, *ob = out_off + x.base;
  t.i0 = ib[x.a0];
  t.i1 = lo32(ib, x.a1);
  load_end<kGaps>(t, in_end, s, L1, lane);
  t.o0 = ob[x.a0];
  t.o1 = lo32(ob, x.a1);
  t.ie = ib[x.ae];
  t.oe = ob[x.ae];
}

// The two halves of load_off, for the launch's opening.
template <bool kGaps>
__device__ __forceinline__ void load_off_in(TileOff &t, const uint64_t *__restrict__ in_off,
                                            const uint32_t *__restrict__ in_end, uint64_t s, uint64_t L1,
                                            uint32_t tl, uint32_t lane) {
  const TileIdx x(s, L1, tl, lane);
  const uint64_t *ib = in_off + x.base;
  t.i0 = ib[x.a0];
  t.i1 = lo32(ib, x.a1);
  load_end<kGaps>(t, in_end, s, L1, lane);
  t.ie = ib[x.ae];
}
__device__ __forceinline__ void load_off_out(TileOff &t, const uint64_t *__restrict__ out_off, uint64_t s,
                                             uint64_t L1, uint32_t tl, uint32_t lane) {
  const TileIdx x(s, L1, tl, lane);
  const uint64_t *ob = out_off + x.base;
  t.o0 = ob[x.a0];
  t.o1 = lo32(ob, x.a1);
  t.oe = ob[x.ae];
}

struct TileIn {
  u32x4 v[kPF];
};

// Input chunks [0, kPF*64) from the 16-B aligned start of a tile whose input
// is [ib, iend) in in_off units (chunk indices clamped; nothing for an empty
// range, whose aligned chunk may lie past the buffer).
// `keep` (the opening): the chunk indices come back, for the caller to keep
// live until the loads have landed (a register that addressed a load still in
// flight and is then overwritten makes the compiler wait for the load).
__device__ __forceinline__ void load_in(TileIn &t, const uint8_t *__restrict__ in, uint64_t in_bias, uint64_t ib,
                                        uint64_t iend, uint32_t lane, uint32_t *keep = nullptr) {
  // (nothing for an empty or reversed range: literals out of order -- the
  // framed strings of read_strings may be -- give iend < ib, and such a tile
  // is never staged; loading from ib would read past the buffer's end)
  if (iend <= ib) return;
  const uint8_t *a = in + (ib - in_bias);
  const uint32_t delta = (uint32_t)((uintptr_t)a & 15u);
  const u32x4 *src = (const u32x4 *)(a - delta);
  const uint64_t need = ((iend - ib) + delta + 15u) >> 4;
  const uint32_t chunks = (uint32_t)min(need, (uint64_t)(kWIn / 16));
  CRUMB(52, src + min(lane + (uint32_t)kWave * (kPF - 1), chunks - 1u));
#pragma unroll
  for (int k = 0; k < kPF; k++) {
    const uint32_t c = min(lane + (uint32_t)kWave * k, chunks - 1u);
    t.v[k] = __builtin_nontemporal_load(src + c);  // aligned, holds a valid byte: never crosses a page
    if (keep) keep[k] = c;
  }
}

__device__ __forceinline__ void put_chunk(WaveSmem &ws, uint32_t c, u32x4 v) {
  v.x = __builtin_bswap32(v.x);
  v.y = __builtin_bswap32(v.y);
  v.z = __builtin_bswap32(v.z);
  v.w = __builtin_bswap32(v.w);
  *(u32x4 *)(ws.in_w + 4u * c) = v;
}

// read_strings' outcome of a decoded string (hc/io.go:92-96), applied where
// the decode writes it when `str_kind` (the framed strings' kinds) is given:
// INVALID keeps length 0; a Huffman string that decoded to nothing is io.EOF.
// (Raw and unreadable strings are empty literals here: 0 / OK, as the
// reference returns for the unreadable ones; raw payloads are the finish
// pass's.)
constexpr uint32_t kStrEof = 2;      // MHQ_STR_EOF (include/mhq_huff.h)
constexpr uint32_t kStrNoSpace = 3;  // MHQ_STR_NOSPACE
__device__ __forceinline__ void str_outcome(const uint8_t *__restrict__ str_kind, uint64_t i, uint32_t &len,
                                            uint32_t &st) {
  if (st != 0u)
    len = 0;
  else if (len == 0u && (str_kind[i] & 3u) == 1u)
    st = kStrEof;
}

// out_len / status of literals [s, s + m) from the wave's len array (streaming
// stores: config 2 37.1 -> 35.7 us, config 3 32.9 -> 31.8).
__device__ __forceinline__ void flush_lens(const WaveSmem &ws, uint64_t s, uint32_t m, uint32_t *__restrict__ out_len,
                                           uint8_t *__restrict__ status, uint32_t lane,
                                           const uint8_t *__restrict__ str_kind = nullptr) {
#pragma unroll
  for (int h = 0; h < 2; h++) {
    const uint32_t j = lane + (uint32_t)kWave * h;
    if (j < m) {
      const uint32_t v = ws.len[j];
      uint32_t len = v & 0x7fffffffu, st = v >> 31;
      if (str_kind) str_outcome(str_kind, s + j, len, st);
      __builtin_nontemporal_store(len, out_len + s + j);
      __builtin_nontemporal_store((uint8_t)st, status + s + j);
    }
  }
}

// A wave's loop priority: with every loop at one priority the SIMD issues
// oldest-first, so a SIMD's three waves finish their equal work one after the
// other and the last runs alone (the age staircase).  The loops
// of a wave's first two tiles run at priority 1, the rest at 0, so the younger
// waves catch up at every tile boundary (-1 to -2 % on every shape).
__device__ __forceinline__ void set_loop_prio(uint32_t p) {
  if (p)
    __builtin_amdgcn_s_setprio(1);
  else
    __builtin_amdgcn_s_setprio(0);
}

// Decodes the m literals whose boundary records rec[0..m] and input bytes are
// staged: zero the output region, sort, decode into out_w / len.
template <bool kGaps>
__device__ __forceinline__ void decode_piece(const Smem &sm, WaveSmem &ws, uint32_t m, uint32_t out_bytes,
                                             uint32_t lane, [[maybe_unused]] int tls = -1, uint32_t prio = 0) {
  // masked steps per end test: 3 for the plain decode (north star -2.7 %,
  // config 4 -7 %, print +3 %: profiles/r04c_decode_steps_ab.txt)
  constexpr int kSteps = kGaps ? MHQ_DEC_STEPS_GAPS : MHQ_DEC_STEPS;
  constexpr bool kPair = MHQ_DEC_PAIR;
  for (uint32_t c = lane; c < (out_bytes + 15u) >> 4; c += kWave) *(u32x4 *)(ws.out_w + 4u * c) = u32x4{0u, 0u, 0u, 0u};
  // counting sort by encoded length, longest first
  ws.hist[lane] = 0;
  wave_sync();
  uint32_t key[2], rk[2];
#pragma unroll
  for (int h = 0; h < 2; h++) {
    const uint32_t j = lane + (uint32_t)kWave * h;
    key[h] = 0;
    rk[h] = 0;
    if (j < m) {
      const uint32_t bytes = (kGaps ? ws.len[j] : (ws.rec[j + 1] & 0xffffu)) - (ws.rec[j] & 0xffffu);
      const uint32_t bk = bytes < 48u ? bytes : min(48u + ((bytes - 48u) >> 3), (uint32_t)kBuckets - 1u);
      key[h] = (uint32_t)kBuckets - 1u - bk;
      rk[h] = atomicAdd(&ws.hist[key[h]], 1u);
    }
  }
  wave_sync();
  {
    const uint32_t hcount = ws.hist[lane];
    ws.hist[lane] = wave_incl_scan(hcount) - hcount;
  }
  wave_sync();
#pragma unroll
  for (int h = 0; h < 2; h++) {
    const uint32_t j = lane + (uint32_t)kWave * h;
    if (j < m) ws.order[ws.hist[key[h]] + rk[h]] = (uint8_t)j;
  }
  wave_sync();
  // Lane t decodes rank t, then rank 127 - t if there is one: the 64 longest
  // literals one per lane, the rest on the lanes with the shortest of those
  // (LPT).  The lane's two fast loops run back to back in one loop (it moves
  // to its second literal in place), so lanes stay busy until all are done.
  const bool hasA = lane < m, hasB = 2u * kWave - 1u - lane < m;
  LitRef<kGaps> A, B;
  A.load(ws, hasA ? ws.order[lane] : 0u);
  B.load(ws, hasB ? ws.order[2u * kWave - 1u - lane] : 0u);
  const uint32_t ostartA = A.optr, ostartB = B.optr;
#ifdef MHQ_DBG_BOUNDS
  {
    const uint32_t span = (ws.rec[m] & 0xffffu) * 8u;  // the staged input's end (bits)
    if (hasA) {
      DBG_CHECK(A.p <= A.endbit && A.endbit <= span, 2, A.p | (uint64_t)A.endbit << 32, span);
      DBG_CHECK(A.optr <= A.oend && A.oend <= out_bytes, 3, A.optr | (uint64_t)A.oend << 32, out_bytes);
    }
    if (hasB) {
      DBG_CHECK(B.p <= B.endbit && B.endbit <= span, 2, B.p | (uint64_t)B.endbit << 32, span);
      DBG_CHECK(B.optr <= B.oend && B.oend <= out_bytes, 3, B.optr | (uint64_t)B.oend << 32, out_bytes);
    }
    DBG_CHECK(out_bytes <= (uint32_t)kWOut, 4, out_bytes, m);
  }
#endif
  TL(tls);
  set_loop_prio(prio);
  // Every literal runs the masked loop to its end (ones past the end: no end
  // test, no separate tail loop); the lane moves from A to B in place.  A
  // literal with a code across its end (not well formed) takes the checked
  // loop.  So does a piece in which a literal whose region can truncate
  // (under floor(8 bits / 5) bytes) turned out not to fit it (below): regions
  // sized to the exact plaintext -- a caller that knows the lengths, as every
  // round trip does -- stay on the fast loop.
  constexpr uint32_t kRedo = 0xffffffffu;
  const bool roomA = hasA && (A.roomy() || A.in_slice());
  const bool roomB = hasB && (B.roomy() || B.in_slice());
  uint32_t rA = kRedo, rB = kRedo;
  {
    WinBuf3 in;
    in.init(ws.in_w, roomA ? A.p : B.p, roomA ? A.endbit : B.endbit);
    OutAccL out;
    out.init(ws.out_w, roomA ? A.optr : B.optr);
    uint32_t ost = roomA ? ostartA : ostartB;
    PendL pend{out.op, 0u};
    bool onB = !roomA, active = roomA || roomB;
    while (active) {
      bool stop;
      // kSteps steps per end test: a finished literal (EOS prefix, or a code
      // across its end) stays finished through further steps (no bits
      // consumed at the EOS prefix; `left` stays negative), so the last
      // step's result covers them all; only that step resolves codes of 13+
      // bits through LUT2 (the others leave them, consuming nothing)
      // (kPair: the steps go in pairs on one window read, an odd one last:
      // north star -3.6 %, config 2 -4 %, config 3 -2 %, print -2 %,
      // profiles/r05u_decode_pair_ab.txt)
      bool fin;
      if constexpr (kPair) {
#pragma unroll
        for (int k = 0; k + 2 < kSteps; k += 2) win_pair<false>(sm, in, out, pend, stop);
        if constexpr (kSteps % 2 == 0)
          fin = win_pair<true>(sm, in, out, pend, stop);
        else
          fin = win_step32<true>(sm, in, out, pend, stop);
      } else {
#pragma unroll
        for (int k = 1; k < kSteps; k++) win_step32<false>(sm, in, out, pend, stop);
        fin = win_step32<true>(sm, in, out, pend, stop);
      }
      if (fin) {
        // stop: the EOS prefix (INVALID when a 31st bit of the literal
        // follows); left < 0: a code crossed the end (the piece is redone)
        const uint32_t r = in.left < 0 ? kRedo : (out.optr(ws.out_w) - ost) | ((uint32_t)(in.left > kEosOnes) << 31);
        rA = onB ? rA : r;
        rB = onB ? r : rB;
        active = !onB && roomB;
        in.init(ws.in_w, B.p, B.endbit);
        out.init(ws.out_w, B.optr);
        ost = ostartB;
        onB = true;
      }
      DBG_CHECK((uint32_t)(pend.p - ws.out_w) < (uint32_t)kWOut / 4u + 4u, 1, pend.p - ws.out_w, kSteps);
    }
    atomicOr(pend.p, pend.v);
  }
  // a lane that ran a literal through the fast loop and got no result crossed its end
  const bool crossed = (roomA && rA == kRedo) || (roomB && rB == kRedo);
  {
    // A fast result for a region that can truncate stands when it fits: a
    // longer output has run past the region into a neighbour's bytes, and an
    // INVALID literal that fills its region exactly is OK to the reference
    // (Read returns once its buffer is full, hc/huffman.go:104, before the
    // bits after).  Otherwise the whole piece is decoded again by the checked
    // loop over a re-zeroed output region.
    auto overflow = [](const LitRef<kGaps> &L, uint32_t r) {
      const uint32_t len = r & 0x7fffffffu, region = L.oend - L.optr;
      return r != kRedo && !L.roomy() && (len > region || (len == region && (r >> 31)));
    };
    // (a redo must see this piece's records intact: in_slice kept every write
    // inside out_w)
    const bool badA = hasA && overflow(A, rA);
    const bool badB = hasB && overflow(B, rB);
    if (__ballot(badA || badB || crossed)) {
      wave_sync();
      for (uint32_t c = lane; c < (out_bytes + 15u) >> 4; c += kWave) *(u32x4 *)(ws.out_w + 4u * c) = u32x4{0u, 0u, 0u, 0u};
      wave_sync();
      rA = kRedo;
      rB = kRedo;
    }
  }
  TL(tls < 0 ? -1 : tls + 1);
  if (hasA) ws.len[A.lit] = rA != kRedo ? rA : decode_checked_k<kGaps>(sm, ws, A.p, A.endbit, A.optr, A.oend);
  if (hasB) ws.len[B.lit] = rB != kRedo ? rB : decode_checked_k<kGaps>(sm, ws, B.p, B.endbit, B.optr, B.oend);
  wave_sync();
}

// ---- oversized tiles: literals streamed through per-lane windows ----------
// A tile whose bytes exceed the slices (long literals: config 4's Zipf tail,
// config 5's 438-byte literals) is decoded with every lane on a literal of its
// own (lane l: literals l, l + 64), in wave-wide rounds.  Each round a lane
// stages the next 128 B of its literal (from the 16-B chunk holding its bit
// position) into a private LDS window — the windows reuse the wave's input
// and output slices — and runs probes (long_step) until its window runs low
// or its literal ends; the end runs the checked loop (the reference's end and
// INVALID rules).  Output goes straight to global memory from the register
// accumulator (OutAccG), which lives across rounds.  Literals whose output
// region truncates are decoded by their lane with decode_literal_global.

#ifndef MHQ_DEC_LONGW  // a lane's window in words (multiple of 4)
#define MHQ_DEC_LONGW 32
#endif
constexpr uint32_t kLongWords = MHQ_DEC_LONGW;  // a lane's window: 128 B, 8 aligned 16-B chunks
static_assert(sizeof(uint32_t) * kLongWords * kWave <= sizeof(uint32_t) * (kWIn / 4 + 4 + kWOut / 4 + 4),
              "the lanes' windows fit the wave's slices");

// Output bytes in registers, stored straight to global memory: `acc` holds
// the bytes from word ow of the literal's 4-B aligned output base up, `ab`
// bits of it decided.  Completed words inside the literal's region collect in
// q0..q3 and leave as one aligned 16-B store per four (a lane's stores are
// scattered over the wave's literals, so each store instruction touches 64
// lines: four times fewer of them matters more than their width); words of a
// 16-B group the region does not own whole leave as dword stores.  The first
// word of a region that starts mid-word is shared with the previous
// literal's region, so it is kept in `first` and finish() writes its bytes one
// by one, as it does the decided bytes of the last word.
// kPend (decode_long_kernel: 2): completed 16-B groups wait in up to kPend
// slots (a third one in a round is stored at once) for drain(), which the
// streamed loop calls for the whole wave right after a window refill: one
// store instruction then carries most lanes' groups instead of the few lanes
// that complete a group on a given step, and no store is in flight when the
// next refill waits on vmcnt.  The stores cost config 5 31 % of the kernel
// (1272 against 878 us without them; where they land made no difference,
// profiles/r06/r06vx_*); this takes back 5 % (1274 -> 1211-1213 us; drains
// every 8 steps instead: 1243; four slots: 1226).
template <int kPend>
struct OutAccGT {
  static_assert(kPend >= 0 && kPend <= 4, "pending groups: up to four");
  uint64_t acc;
  uint32_t ow, ab, owf, first, rs, ga, q0, q1, q2, q3;
  uint32_t np;
  uint32_t pa[kPend > 0 ? kPend : 1];
  u32x4 pg[kPend > 0 ? kPend : 1];  // (registers: indexed by constants only)
  // optr: the region's start from the 4-B aligned base gout; ga: gout's word
  // position in its 16-B group ((gout / 4) % 4), so word x sits at word
  // x + ga of the 16-B grid
  __device__ __forceinline__ void init(uint32_t optr, uint32_t ga_ = 0) {
    ga = ga_;
    acc = 0;
    ow = optr >> 2;
    ab = (optr & 3u) * 8u;
    owf = (optr + 3u) >> 2;  // the first word owned whole
    first = 0;
    rs = optr;
    q0 = q1 = q2 = q3 = 0;
    np = 0;
  }
  __device__ __forceinline__ void put(uint32_t syms, uint32_t nbits) {
    acc |= (uint64_t)syms << ab;
    ab += nbits;
  }
  // the 16-B group of word x is owned whole: all four words at or past owf
  __device__ __forceinline__ bool grouped(uint32_t x) const { return ((x + ga) & ~3u) >= owf + ga; }
  __device__ __forceinline__ void flush(uint32_t *gout) {
    const bool full = ab >= 32u;
    const uint32_t v = (uint32_t)acc;
    if (full && ow >= owf) {
      CRUMB(53, gout + ow);
      if (!grouped(ow)) {
        if (DBG_OK(dbg_out_ok(gout + ow, 4), 23, gout + ow, ow)) gout[ow] = v;
      } else {
        const uint32_t r = (ow + ga) & 3u;
        q0 = r == 0u ? v : q0;
        q1 = r == 1u ? v : q1;
        q2 = r == 2u ? v : q2;
        q3 = r == 3u ? v : q3;
        if (kPend && r == 3u && np < (uint32_t)kPend) {  // (the group waits for drain)
#pragma unroll
          for (int k = 0; k < kPend; k++) {
            const bool here = np == (uint32_t)k;
            pg[k] = here ? u32x4{q0, q1, q2, v} : pg[k];
            pa[k] = here ? ow - 3u : pa[k];
          }
          np++;
        } else if (r == 3u && DBG_OK(dbg_out_ok(gout + ow - 3u, 16), 24, gout + ow - 3u, ow)) {
          *(u32x4 *)(gout + ow - 3u) = u32x4{q0, q1, q2, v};
        }
      }
    }
    first = (full && ow < owf) ? v : first;
    acc >>= ab & 32u;
    ow += ab >> 5;
    ab &= 31u;
  }
  // the pending groups leave (the wave's lanes together)
  __device__ __forceinline__ void drain(uint32_t *gout) {
    if (!kPend) return;
#pragma unroll
    for (int k = 0; k < kPend; k++)
      if (np > (uint32_t)k && DBG_OK(dbg_out_ok(gout + pa[k], 16), 24, gout + pa[k], pa[k])) *(u32x4 *)(gout + pa[k]) = pg[k];
    np = 0;
  }
  __device__ __forceinline__ void finish(uint32_t *gout) {
    flush(gout);
    drain(gout);
    // whole words of the last, incomplete 16-B group
    CRUMB(54, gout + ow);
    if (grouped(ow)) {
      const uint32_t r = (ow + ga) & 3u, g = ow - r;
      if (DBG_OK(dbg_out_ok(gout + g, 4 * r), 25, gout + g, r)) {
        if (r > 0u) gout[g] = q0;
        if (r > 1u) gout[g + 1u] = q1;
        if (r > 2u) gout[g + 2u] = q2;
      }
    }
    uint8_t *g8 = (uint8_t *)gout;
    const uint32_t hi = ab >> 3, lo = ow < owf ? (rs & 3u) : 0u;
    if (ow >= owf && (rs & 3u)) {
      for (uint32_t x = rs & 3u; x < 4u; x++)
        if (DBG_OK(dbg_out_ok(g8 + (owf - 1u) * 4u + x, 1), 26, g8 + (owf - 1u) * 4u + x, rs))
          g8[(owf - 1u) * 4u + x] = (uint8_t)(first >> (8u * x));
    }
    for (uint32_t x = lo; x < hi; x++)
      if (DBG_OK(dbg_out_ok(g8 + ow * 4u + x, 1), 27, g8 + ow * 4u + x, ow)) g8[ow * 4u + x] = (uint8_t)(acc >> (8u * x));
  }
  __device__ __forceinline__ uint32_t optr() const { return ow * 4u + (ab >> 3); }
};
using OutAccG = OutAccGT<0>;

// The checked loop of decode_checked on a window, with the lane's running
// accumulator (roomy literals only: no buffer-full rule).  Returns the status.
template <class BB, class SM, class Acc>
__device__ __forceinline__ uint32_t end_checked_g(const SM &sm, const uint32_t *win, uint32_t p, uint32_t endbit,
                                                  Acc &out, uint32_t *gout, uint32_t swz) {
  BB in;
  in.init(win, p, swz);
  uint32_t bad = 0;
  bool fin = false;
  while (!fin) {
    in.refill();
    const uint32_t w = in.top32();
    const uint32_t left = endbit - in.p;
    const uint32_t e = sm.lut1[w >> (32 - kLut1Bits)];
    uint32_t tot = e & 0xffu, ns8 = (e >> 8) & 0xffu, syms = e >> 16, len0 = sm.clen[(e >> 16) & 0xffu];
    if (e == 0) {
      const uint32_t L = long_code(sm.lut2, w, syms);
      len0 = tot = L ? L : 0xffffffffu;
      ns8 = 8u;
      bad |= L == 0 && left > (uint32_t)kEosOnes;
    }
    const uint32_t c8 = tot <= left ? ns8 : (len0 <= left ? 8u : 0u);
    const uint32_t cons = c8 == 16u ? tot : (c8 ? len0 : 0u);
    out.put(__builtin_amdgcn_ubfe(syms, 0, c8), c8);
    in.bb <<= cons & 63u;
    in.p += cons;
    fin = c8 == 0;
    out.flush(gout);
  }
  return bad;
}

// One probe of the stream path: a long code (or the EOS prefix) found by the
// probe is resolved at once through LUT2 — long literals are where long
// codes pile up (config 5 has nothing else), and the fast step would spend a
// second LUT1 probe finding it again.  Same end rules as decode_checked.
template <class Acc, class BB, bool kFlush = true, class SM = Smem>
__device__ __forceinline__ void long_step(const SM &sm, uint32_t *otgt, BB &in, Acc &out, uint32_t endbit,
                                          int &lim, uint32_t &bad) {
  // Branch free: LUT1 and LUT2 are read together (independent addresses, one
  // LDS round trip) and the entry is selected after.  kLongOnes or more
  // leading ones can only start a code longer than LUT1's reach, or the EOS
  // prefix (c >= 30, LUT2's row clamped to 29 then, its entry unused).
  const uint32_t top = in.top32();
  const uint32_t nw = ~top;
  const uint32_t c = nw ? (uint32_t)__builtin_clz(nw) : 32u;
  const uint32_t cc = min(c, (uint32_t)kEosOnes - 1u);
  const uint32_t e2 = sm.lut2[(cc << kLut2SubBits) | ((top << (cc + 1u)) >> (32 - kLut2SubBits))];
  const uint32_t e1r = sm.lut1[top >> (32 - kLut1Bits)];
  const uint32_t e1 = c >= (uint32_t)kLongOnes ? 0u : e1r;
  const uint32_t L = c >= (uint32_t)kEosOnes ? 0u : e2 >> 8;
  const uint32_t left = endbit - in.p;
  const bool lng = e1 == 0u;
  // a long code past the end, or the EOS prefix: the literal ends here, INVALID
  // when a 31st bit exists (nil child, hc/huffman.go:111-113)
  const bool stop = lng && (L == 0u || L > left);
  bad = stop ? (uint32_t)(L == 0u && left > (uint32_t)kEosOnes) : bad;
  lim = stop ? -1 : lim;
  const uint32_t e = lng ? (stop ? 0u : (L | (8u << 8) | ((e2 & 0xffu) << 16))) : e1;
  out.put(e >> 16, (e >> 8) & 0xffu);
  in.consume(e);
  in.refill();
  if (kFlush) out.flush(otgt);
}

// (decode_tile_long_body: always inlined -- the long-literal kernel's
// register budget applies to it; decode_tile_long: the decode kernels' call,
// inlined or not at the compiler's choice)
template <bool kGaps, class SM, class W, uint32_t kW = kLongWords, int kPend = 0>
__device__ __forceinline__ void decode_tile_long_body(const SM &sm, W &ws, const uint8_t *__restrict__ in,
                                 const uint64_t *__restrict__ in_off, const uint32_t *__restrict__ in_end,
                                 uint64_t in_bias, uint8_t *__restrict__ out,
                                 const uint64_t *__restrict__ out_off, uint64_t out_bias,
                                 uint32_t *__restrict__ out_len, uint8_t *__restrict__ status, uint64_t s,
                                 uint32_t cnt, uint32_t lane, const uint8_t *__restrict__ str_kind = nullptr) {
  // (W: the wave's LDS, whose in_w starts the windows: in the decode kernel
  // they span the wave's input and output slices)
  // (kW: the window's words, 32 or 16; kCpw of its 16-B chunks)
  constexpr uint32_t kCpw = kW / 4u;
  static_assert(kW == 32u || kW == 16u, "window of 8 or 4 chunks");
  uint32_t *win = ws.in_w + lane * kW;
  const uint32_t swz = (lane % kCpw) << 2;  // BitBufS: the window's chunk swizzle
  constexpr uint32_t kWinBits = kW * 32u;
  constexpr uint32_t kSafe = kWinBits - 96u;  // fast steps stay below: 24 bits + two words of look-ahead
  uint32_t j = lane;
  bool have = false;
  uint64_t ib = 0, ie = 0, ob = 0;
  uint64_t rel = 0;  // bits of the literal consumed
  uint32_t *gout = nullptr;
  OutAccGT<kPend> acc;
  acc.init(0);
  uint32_t ostart = 0;
  [[maybe_unused]] uint64_t oreg = 0;  // the literal's region (bytes; MHQ_DBG_BOUNDS)
  // next literal of this lane (roomy ones stay; the rest are done at once from global memory)
  auto next_lit = [&]() {
    have = false;
    while (j < cnt) {
      CRUMB(55, in_off + s + j);
      ib = in_off[s + j];
      if (kGaps) {  // the end's low word: the end is the first at or after ib with it
        const uint32_t e = in_end[s + j];
        ie = (ib & ~0xffffffffull) | e;
        if (e < (uint32_t)ib) ie += 1ull << 32;
      } else {
        ie = in_off[s + j + 1];
      }
      CRUMB(56, out_off + s + j + 1);
      ob = out_off[s + j];
      const uint64_t oe = out_off[s + j + 1];
      uint8_t *o = out + (ob - out_bias);
      CRUMB(57, out_len + s + j);
      if (ie == ib) {  // nothing to read: Read at EOF
        uint32_t len = 0, st = 0;
        if (kGaps && str_kind) str_outcome(str_kind, s + j, len, st);
        out_len[s + j] = len;
        status[s + j] = (uint8_t)st;
      } else if (oe - ob < (ie - ib) * 8u / 5u) {  // a truncating region: the exact slow path
        decode_literal_global(in + (ib - in_bias), ie - ib, o, oe - ob, sm, out_len + s + j, status + s + j);
      } else {
        gout = (uint32_t *)(o - ((uintptr_t)o & 3u));  // pointer arithmetic keeps it global: no flat stores
        ostart = (uint32_t)((uintptr_t)o & 3u);
        acc.init(ostart, (uint32_t)((uintptr_t)gout >> 2) & 3u);
        oreg = oe - ob;
        rel = 0;
        have = true;
        return;
      }
      j += kWave;
    }
  };
  next_lit();
  while (__ballot(have)) {
    // stage: the 8 aligned chunks from the one holding the lane's bit position
    // (the last one holding a byte of the literal at most), by LDS-DMA: wave
    // instruction k loads the windows of lanes 8k..8k+7, 8 lanes a window, so
    // each instruction reads 8 whole 128-B runs instead of 16 B of 64 runs;
    // window bytes stay in memory order (BitBufS swaps on read)
    uint32_t p = 0, endw = 0, nck = 0;
    uint64_t src = 0;
    if (have) {
      const uint8_t *a = in + (ib - in_bias) + (rel >> 3);
      const uint32_t delta = (uint32_t)((uintptr_t)a & 15u);
      const uint8_t *a16 = a - delta;
      src = (uint64_t)(uintptr_t)a16;
      const uint8_t *last = in + (ie - in_bias) - 1;  // the literal's last byte
      DBG_CHECK(a <= last, 8, rel, ie - ib);
      nck = min((uint32_t)(((uintptr_t)last - (uintptr_t)a16) >> 4) + 1u, kCpw);
      p = delta * 8u + (uint32_t)(rel & 7u);
      endw = p + (uint32_t)((ie - ib) * 8u - rel);  // the literal's end in window bits (may lie beyond)
    }
#pragma unroll
    for (uint32_t k = 0; k < kCpw; k++) {
      // slot lane % kCpw of owner o's window takes chunk (lane % kCpw) ^ (o % kCpw)
      const uint32_t o = (kWave / kCpw) * k + lane / kCpw, c = (lane % kCpw) ^ (o % kCpw);
      const uint64_t so = (uint64_t)__shfl((unsigned long long)src, (int)o);
      const uint32_t no = (uint32_t)__shfl((int)nck, (int)o);
      if (c < no) CRUMB(58, so + 16u * c);
      if (c < no && DBG_OK(dbg_in_ok((const void *)(uintptr_t)(so + 16u * c), 16), 29, so + 16u * c, no))  // chunks past the literal's last one stay unloaded: their bits are never consumed
        __builtin_amdgcn_global_load_lds((g_void *)(uintptr_t)(so + 16u * c), (lds_void *)(ws.in_w + 256u * k), 16, 0,
                                         0);
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    wave_sync();
    // the previous round's groups leave now that the window loads are in:
    // stores issued just before a refill would hold up its vmcnt wait (gfx9
    // counts stores in vmcnt), and one store carries most lanes' groups
    acc.drain(gout);
    if (have) {
      const bool ends_here = endw + 64u <= kWinBits;
      BitBufS bin;
      bin.init(win, p, swz);
      uint32_t bad = 0;
      const int lim0 = ends_here ? (int)endw - 24 : (int)kSafe;
      int lim = lim0;
      // two probes per flush while two codes (<= 30 bits each) surely fit,
      // then single ones up to the end test's bound
      const int lim2 = lim0 - 30;
      while ((int)bin.p <= lim2 && lim != -1) {
        long_step<OutAccGT<kPend>, BitBufS, false>(sm, gout, bin, acc, endw, lim, bad);
        if (lim != -1) long_step<OutAccGT<kPend>, BitBufS, false>(sm, gout, bin, acc, endw, lim, bad);
        acc.flush(gout);
      }
      while ((int)bin.p <= lim) long_step(sm, gout, bin, acc, endw, lim, bad);
      const bool stopped = lim == -1 && lim0 != -1;  // a fast step finished the literal (EOS prefix, long code past the end)
      if (stopped || ends_here) {
        const uint32_t st = stopped ? bad : end_checked_g<BitBufS>(sm, win, bin.p, endw, acc, gout, swz);
        uint32_t got = acc.optr() - ostart, st2 = st;
        DBG_CHECK(got <= oreg, 6, got, oreg);
        acc.finish(gout);
        CRUMB(59, out_len + s + j);
        if (kGaps && str_kind) str_outcome(str_kind, s + j, got, st2);
        out_len[s + j] = got;
        status[s + j] = (uint8_t)st2;
        j += kWave;
        next_lit();
      } else {
        rel += bin.p - p;
      }
    }
    wave_sync();  // every lane is done reading its window (look-ahead reads reach the neighbour's)
  }
}
template <bool kGaps, class SM, class W>
__device__ MHQ_CALLEE_LONG void decode_tile_long(const SM &sm, W &ws, const uint8_t *__restrict__ in,
                                                 const uint64_t *__restrict__ in_off,
                                                 const uint32_t *__restrict__ in_end, uint64_t in_bias,
                                                 uint8_t *__restrict__ out, const uint64_t *__restrict__ out_off,
                                                 uint64_t out_bias, uint32_t *__restrict__ out_len,
                                                 uint8_t *__restrict__ status, uint64_t s, uint32_t cnt, uint32_t lane,
                                                 const uint8_t *__restrict__ str_kind = nullptr) {
  decode_tile_long_body<kGaps>(sm, ws, in, in_off, in_end, in_bias, out, out_off, out_bias, out_len, status, s, cnt,
                               lane, str_kind);
}

// Slow path: a tile whose bytes exceed the slices, in greedy pieces staged
// synchronously from global memory; a literal larger than a slice alone is
// decoded by lane 0 from global memory.
[[maybe_unused]] __device__ void decode_tile_pieces(const Smem &sm, WaveSmem &ws, const uint8_t *__restrict__ in,
                                   const uint64_t *__restrict__ in_off, uint64_t in_bias, uint8_t *__restrict__ out,
                                   const uint64_t *__restrict__ out_off, uint64_t out_bias,
                                   uint32_t *__restrict__ out_len, uint8_t *__restrict__ status, uint64_t s,
                                   uint32_t cnt, uint32_t lane) {
  uint32_t cur = 0;
  while (cur < cnt) {
    const uint64_t ib = uniform64(in_off[s + cur + vzero()]), ob = uniform64(out_off[s + cur + vzero()]);
    const uint8_t *ia = in + (ib - in_bias);
    uint8_t *oa = out + (ob - out_bias);
    const uint32_t idelta = (uint32_t)((uintptr_t)ia & 15u), odelta = (uint32_t)((uintptr_t)oa & 15u);
    // longest prefix [cur, cur + m) that fits both slices (the test is monotone
    // in the literal index, so the count of fitting literals is that length)
    uint32_t m = 0;
#pragma unroll
    for (int h = 0; h < 2; h++) {
      const uint32_t j = cur + lane + (uint32_t)kWave * h;  // literal j ends at offset index j + 1
      const bool ok = j < cnt && (in_off[s + j + 1] - ib) + idelta <= (uint64_t)kWIn &&
                      (out_off[s + j + 1] - ob) + odelta <= (uint64_t)kWOut;
      m += popc64(__ballot(ok));
    }
    if (m == 0) {
      if (lane == 0) {
        const uint64_t ie = in_off[s + cur + 1], oe = out_off[s + cur + 1];
        decode_literal_global(ia, ie - ib, oa, oe - ob, sm, out_len + s + cur, status + s + cur);
      }
      cur += 1;
      continue;
    }
#pragma unroll
    for (int h = 0; h < 3; h++) {
      const uint32_t j = lane + (uint32_t)kWave * h;
      if (j <= m) {
        const uint64_t ij = in_off[s + cur + j], oj = out_off[s + cur + j];
        ws.rec[j] = (uint32_t)(ij - ib + idelta) | (uint32_t)(oj - ob + odelta) << 16;
      }
    }
    wave_sync();
    const uint32_t in_bytes = ws.rec[m] & 0xffffu, out_bytes = ws.rec[m] >> 16;
    stage_in<true, false>(ws.in_w, kWIn / 4, ia - idelta, in_bytes, lane);
    wave_sync();
    decode_piece<false>(sm, ws, m, out_bytes, lane);
    store_out_batched<kOutRounds>(oa - odelta, (const uint8_t *)ws.out_w, odelta, out_bytes, lane);
    flush_lens(ws, s + cur, m, out_len, status, lane);
    wave_sync();
    cur += m;
  }
}

// kGaps: literal i is in[in_off[i] .. in_end[i]), in_end[i] <= in_off[i + 1]
// (the bytes between belong to no literal: the Huffman payloads of a block of
// framed string fields, read where they lie).  A tile is staged only when its
// literals are in that order and fit; every other tile streams (decode_tile_long,
// any order, overlaps included).  The staged tile keeps each literal's end in
// its len slot until the results overwrite it.
template <bool kGaps>
__device__ __forceinline__ void decode_body(Smem &sm, const uint8_t *__restrict__ in,
                                            const uint64_t *__restrict__ in_off,
                                            const uint32_t *__restrict__ in_end, const StrFinish &str,
                                            uint64_t in_bias, uint64_t n, uint8_t *__restrict__ out,
                                            const uint64_t *__restrict__ out_off, uint64_t out_bias,
                                            uint32_t *__restrict__ out_len, uint8_t *__restrict__ status,
                                            const uint32_t *__restrict__ g_lut1, const uint16_t *__restrict__ g_lut2,
                                            const uint8_t *__restrict__ g_len, uint64_t per_block, uint32_t tl0) {
  const uint32_t tid = threadIdx.x;
  const uint32_t lane = tid % kWave;
  const uint32_t wave = tid / kWave;
  const uint64_t L0 = (uint64_t)blockIdx.x * per_block;
  if (L0 >= n) return;
  const uint64_t L1 = min(L0 + per_block, n);
  WaveSmem &ws = sm.w[wave];
  TL(0);

  // Workgroup b owns literals [L0, L1), in tiles of tl literals.  Wave w takes
  // tiles w, w + kWaves, w + 2 kWaves, then claims from the LDS counter, three
  // tiles ahead of the one it decodes.
  uint32_t tile = wave, tile2 = tile + kWaves, tile3 = tile + 2 * kWaves;
  TileOff off, off2;
  // The opening is bound by the bytes every CU loads at once (all of them do),
  // so loads go in the order they are needed: the batch's boundary offsets
  // (the tile-length test below), the first tile's input offsets, its input,
  // then its output offsets, the tables and the second tile's offsets.
  // (Every wave loads them, as scalar loads, and waits for them only where
  // they are used: a load under `tid == 0` waited at once.)
  const bool local = kGaps && str.local;  // (uniform)
  const uint64_t bnd[4] = {in_off[local ? L1 : n], in_off[local ? L0 : 0], out_off[local ? L1 : n],
                           out_off[local ? L0 : 0]};
  const uint64_t nb = local ? L1 - L0 : n;
  // read_strings: whether this workgroup finishes its range at the end (its
  // gate word loaded now, used there)
  // (uniform: a scalar value, not a vector pair live across the tile loop --
  // read_fallback_kernel spilled that pair to scratch)
  const uint64_t fin_gate = kGaps && str.finish_needed ? uniform64(__builtin_nontemporal_load(str.finish_needed)) : 0;
  load_off_in<kGaps>(off, in_off, in_end, L0 + (uint64_t)tile * tl0, L1, tl0, lane);
  TileIn tin;
  uint32_t keep[kPF] = {};
  load_in(tin, in, in_bias, uniform64(off.i0), uniform64(off.ie), lane, keep);
  TL(56);  // the first tile's input loads issued
  load_off_out(off, out_off, L0 + (uint64_t)tile * tl0, L1, tl0, lane);
  static_assert(kLut1Size / 4 <= 2 * kT && kLut2Size / 8 <= kT && kT >= 64, "table copy shape");
  // (loads and stores from clamped indices, none under a branch: a load
  // under a branch was waited for inside it, stalling the wave behind its
  // input loads; threads past a table's end store its last chunk again)
  const uint32_t x1 = min(tid + (uint32_t)kT, (uint32_t)(kLut1Size / 4) - 1u);
  const uint32_t x2 = min(tid, (uint32_t)(kLut2Size / 8) - 1u), x3 = tid % 64u;
  const u32x4 tb0 = ((const u32x4 *)g_lut1)[tid];
  const u32x4 tb1 = ((const u32x4 *)g_lut1)[x1];
  const u32x4 tb2 = ((const u32x4 *)g_lut2)[x2];
  const uint32_t tb3 = ((const uint32_t *)g_len)[x3];
  load_off<kGaps>(off2, in_off, in_end, out_off, L0 + (uint64_t)tile2 * tl0, L1, tl0, lane);
  ((u32x4 *)sm.lut1)[tid] = tb0;
  ((u32x4 *)sm.lut1)[x1] = tb1;
  ((u32x4 *)sm.lut2)[x2] = tb2;
  ((uint32_t *)sm.clen)[x3] = tb3;
  if (tid == 0) sm.next_tile = 3 * kWaves;
  // The tile length: the host's tl0 (every wave the same number of tiles)
  // unless the batch's mean literal is too long for tl0 of them to fit the
  // slices, with a 25 % margin; then the most that fit, if that still gives
  // every lane a literal (longer literals keep tl0 and stream).
  if (tid == 0) {
    const uint64_t nin = bnd[0] - bnd[1], nout = bnd[2] - bnd[3];
    const uint64_t ain = (nin + nb - 1) / nb, aout = (nout + nb - 1) / nb;
    // kGaps (read_strings): a 20 % margin, not 25: its means include the
    // frame headers and the scaled regions' slack (config 2: 27.5 and 44 B
    // against 26.5 and 42.4), and a tile length cut below tl0 gives some
    // waves a fourth tile (decode 41.9 against 35.3 us); tile sums of 114
    // literals spread by ~4 %, so 20 % is still five deviations
    const uint64_t fit_in = kGaps ? (uint64_t)(kWIn - 16) * 5u / (6u * ain + 10u)
                                  : (uint64_t)(kWIn - 16) * 4u / (5u * ain + 8u);
    const uint64_t fit_out = kGaps ? (uint64_t)(kWOut - 16) * 5u / (6u * aout + 10u)
                                   : (uint64_t)(kWOut - 16) * 4u / (5u * aout + 8u);
    const uint64_t fit = min(fit_in, fit_out);
    sm.tl = fit >= (uint64_t)kWave && fit < (uint64_t)tl0 ? (uint32_t)fit : tl0;
  }
  __syncthreads();
#pragma unroll
  for (int k = 0; k < kPF; k++) asm volatile("" ::"v"(keep[k]));
  TL(57);  // tables in LDS
  const uint32_t tl = __builtin_amdgcn_readfirstlane(sm.tl);
  if (tl != tl0) {  // the loads above used tl0: again with tl
    load_off<kGaps>(off, in_off, in_end, out_off, L0 + (uint64_t)tile * tl, L1, tl, lane);
    load_off<kGaps>(off2, in_off, in_end, out_off, L0 + (uint64_t)tile2 * tl, L1, tl, lane);
    load_in(tin, in, in_bias, uniform64(off.i0), uniform64(off.ie), lane);
  }
  const uint32_t ntiles = (uint32_t)((L1 - L0 + tl - 1) / tl);
  uint64_t pd_s = 0;  // the previous tile, still in the output slice: literals, output range
  uint32_t pd_m = 0, pd_lo = 0, pd_hi = 0;
  uint8_t *pd_o = nullptr;
  [[maybe_unused]] uint32_t tl_j = 0;

  while (tile < ntiles) {
    const uint64_t s = L0 + (uint64_t)tile * tl;
    const uint32_t cnt = (uint32_t)min((uint64_t)tl, L1 - s);
    const uint64_t ib = uniform64(off.i0), ob = uniform64(off.o0);
    const uint64_t ie = uniform64(off.ie), oe = uniform64(off.oe);
    const uint8_t *ia = in + (ib - in_bias);
    uint8_t *oa = out + (ob - out_bias);
    const uint32_t idelta = (uint32_t)((uintptr_t)ia & 15u), odelta = (uint32_t)((uintptr_t)oa & 15u);
    bool fits = (ie - ib) + idelta <= (uint64_t)kWIn && (oe - ob) + odelta <= (uint64_t)kWOut;
    uint32_t re0 = 0, re1 = 0;  // kGaps: the two literals' ends in the slice
    if (kGaps) {  // staged only if start <= end <= next start for every literal of the tile
      const uint32_t ib32 = (uint32_t)ib - idelta;
      const uint32_t a = (uint32_t)off.i0 - ib32, c = off.i1 - ib32, rie = (uint32_t)ie - ib32;
      re0 = off.e0 - ib32;
      re1 = off.e1 - ib32;
      const uint32_t nx = (uint32_t)__shfl_down((int)a, 1);  // the next lane's first start
      const uint32_t j0 = 2u * lane;
      const bool ok0 = j0 >= cnt || (a <= re0 && re0 <= (j0 + 1u < cnt ? c : rie));
      const bool ok1 = j0 + 1u >= cnt || (c <= re1 && re1 <= (j0 + 2u < cnt ? nx : rie));
      fits = fits && __ballot(!(ok0 && ok1)) == 0;
    }
    __builtin_amdgcn_s_setprio(kPhasePrio);  // staging, flush and sort (serial phases) ahead of other waves' loops
    // claim the tile three ahead (used when this one is done)
    uint32_t tile4 = 0;
    if (lane == 0) tile4 = atomicAdd(&sm.next_tile, 1u);
    if (fits) {  // stage this tile: input words, boundary records
      const uint32_t chunks = (uint32_t)(((ie - ib) + idelta + 15u) >> 4);
#pragma unroll
      for (int k = 0; k < kPF; k++) {
        const uint32_t c = lane + (uint32_t)kWave * k;
        if (c < chunks) put_chunk(ws, c, tin.v[k]);
      }
      const uint32_t j0 = 2u * lane;
      if (j0 < cnt) ws.rec[j0] = (uint32_t)(off.i0 - ib + idelta) | (uint32_t)(off.o0 - ob + odelta) << 16;
      if (j0 + 1u < cnt) ws.rec[j0 + 1] = (off.i1 - (uint32_t)ib + idelta) | (off.o1 - (uint32_t)ob + odelta) << 16;
      if (lane == 0) ws.rec[cnt] = (uint32_t)(ie - ib + idelta) | (uint32_t)(oe - ob + odelta) << 16;
      if (tl_j == 0) TL(58);  // the first tile's input and output offsets arrived
    }
    // the next tile's input (its offsets arrived during the previous decode), the offsets of the one after
    load_in(tin, in, in_bias, uniform64(off2.i0), uniform64(off2.ie), lane);
    off = off2;
    load_off<kGaps>(off2, in_off, in_end, out_off, L0 + (uint64_t)tile3 * tl, L1, tl, lane);
    TL(tl_slot(tl_j, 1));
    // the previous tile's output and lengths leave, then this tile decodes
    if (pd_o) {
      if (DBG_OK(dbg_out_ok(pd_o + pd_lo, pd_hi - pd_lo), 31, pd_o, pd_hi))
        store_out_batched<kOutRounds>(pd_o, (const uint8_t *)ws.out_w, pd_lo, pd_hi, lane);
      flush_lens(ws, pd_s, pd_m, out_len, status, lane, kGaps ? str.kind : nullptr);
    }
    pd_o = nullptr;
    wave_sync();
    TL(tl_slot(tl_j, 2));
    if (fits) {
      if (kGaps) {  // the ends go in the len slots once the previous tile's lengths have left
        const uint32_t j0 = 2u * lane;
        if (j0 < cnt) ws.len[j0] = re0;
        if (j0 + 1u < cnt) ws.len[j0 + 1] = re1;
        wave_sync();
      }
      const uint32_t out_bytes = ws.rec[cnt] >> 16;
      decode_piece<kGaps>(sm, ws, cnt, out_bytes, lane, tl_slot(tl_j, 3), tl_j < 2u ? 1u : 0u);
      pd_o = oa - odelta;
      pd_lo = odelta;
      pd_hi = out_bytes;
      pd_s = s;
      pd_m = cnt;
    } else {
      // a tile a little over the slice (short literals with a few long ones)
      // goes in staged pieces; one of long literals streams through windows
      // (kGaps: every such tile streams)
      if (!kGaps && (ie - ib) <= 2u * (uint64_t)kWIn && (oe - ob) <= 2u * (uint64_t)kWOut)
        decode_tile_pieces(sm, ws, in, in_off, in_bias, out, out_off, out_bias, out_len, status, s, cnt, lane);
      else if constexpr (kGaps)
        decode_tile_long_body<kGaps>(sm, ws, in, in_off, in_end, in_bias, out, out_off, out_bias, out_len, status, s,
                                     cnt, lane, str.kind);
      else
        decode_tile_long<kGaps>(sm, ws, in, in_off, in_end, in_bias, out, out_off, out_bias, out_len, status, s,
                                cnt, lane);
    }
    TL(tl_slot(tl_j, 5));
    tl_j++;
    tile = tile2;
    tile2 = tile3;
    tile3 = __builtin_amdgcn_readfirstlane(tile4);
  }
  if (pd_o) {
    if (DBG_OK(dbg_out_ok(pd_o + pd_lo, pd_hi - pd_lo), 31, pd_o, pd_hi))
      store_out_batched<kOutRounds>(pd_o, (const uint8_t *)ws.out_w, pd_lo, pd_hi, lane);
    flush_lens(ws, pd_s, pd_m, out_len, status, lane, kGaps ? str.kind : nullptr);
  }
  if (kGaps && str.kind) {
    // read_strings' finish of [L0, L1) (hc/io.go:92-96), after every wave's
    // lengths have landed: raw payloads, raw EOFs, cut regions
    const bool clamped = bnd[2] >= str.out_cap;
    if (clamped || fin_gate == str.gen) {  // (uniform)
      __threadfence_block();
      __syncthreads();
      for (uint64_t i = L0 + tid; i < L1; i += kT) {
        const uint8_t kd = str.kind[i];
        if ((kd & 3u) == 2u) continue;  // ReadBit / ReadInt failed: ("", nil), as decoded
        const uint64_t o0 = out_off[i], st0 = str.start[i], nx = str.next[i];
        if (clamped && out_off[i + 1] - o0 < read_cap(kd, st0, str.hend[i], nx)) {
          out_len[i] = 0;  // the region was cut short by the buffer's end
          status[i] = (uint8_t)kStrNoSpace;
        } else if ((kd & 3u) == 0u) {
          const uint64_t take = nx - st0;  // next = start + take (raw)
          if (take == 0 && (kd & kDeclared)) {
            status[i] = (uint8_t)kStrEof;  // the block ended before the payload: io.EOF
          } else if (take) {
            DBG_CHECK(o0 + take <= out_off[i + 1], 13, o0, take);
            if (DBG_OK(dbg_out_ok(out + (o0 - out_bias), take) && dbg_in_ok(str.blk + st0, take), 30, o0, take))
              copy_bytes(out + (o0 - out_bias), str.blk + st0, take);
            out_len[i] = (uint32_t)take;
          }
        }
      }
    }
  }
  TL(63);
}

}  // namespace
}  // namespace mhq
