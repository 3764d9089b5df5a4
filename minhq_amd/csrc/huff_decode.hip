// huff_decode.hip -- gfx950 batch decode of RFC 7541 Huffman literals.
//
// Semantics: hc/huffman.go:102-121 (HuffmanDecompressor.Read, one tree step
// per bit) driven to EOF as Reader.ReadString does (hc/io.go:85-96); see the
// contract in SURVEY.md §8a and the CPU restatement oracle/huff_oracle.c.
//   * every complete code emits its byte; a partial code at the end of the
//     literal (padding or otherwise) is dropped without checks;
//   * 30 one-bits reach the childless node where EOS would be
//     (hc/huffman.go:63-76): one more bit of input is "invalid Huffman coding";
//   * Read stops as soon as its buffer is full (hc/huffman.go:104).
//
// Structure: one workgroup per CU; its waves work independently (no
// workgroup barrier after the table load).  A wave takes a tile of up to 128
// consecutive literals at a time (tiles handed out by an LDS counter) and
// decodes it with two literals per lane:
//   * staging: the tile's offsets and input bytes are loaded into registers
//     one tile ahead (offsets two tiles ahead), so HBM latency hides behind
//     the decode of the current tile.  Input lands in the wave's LDS slice as
//     byte-swapped words (word k = stream bits 32k..32k+31, MSB first); the
//     output is assembled in a zeroed LDS copy of the tile's output region
//     (global layout) and leaves as aligned 16-B stores, with out_len/status
//     as coalesced stores, when the next tile starts;
//   * balance: a counting sort by encoded length (descending) inside the
//     wave; lane t decodes rank t, then rank 127-t, so every lane's two
//     literals add up to about the same length and the 64 lanes of a wave
//     run loops of about the same length;
//   * a literal's bits stream through a 64-bit register buffer refilled one
//     staged word at a time; a probe reads LUT1 with the next 12 bits (one or
//     two codes of <= 12 bits) or, for longer codes, LUT2 by count of leading
//     ones; output bytes gather in a 64-bit register and are OR-ed into the
//     staging one word per step, so literals that share a word need no
//     ordering;
//   * a tile too large for the slices is decoded in pieces that fit; a single
//     literal larger than a slice is decoded by one lane straight from global
//     memory.
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
#ifndef MHQ_DEC_XROUNDS  // tile rounds beyond the fewest that hold the batch (smaller tiles, more of them)
#define MHQ_DEC_XROUNDS 0
#endif
#ifndef MHQ_DEC_PRIO  // wave priority during a tile's staging, flush and sort (0: none)
#define MHQ_DEC_PRIO 3
#endif
#ifndef MHQ_DEC_P3  // a third LUT1 probe per step of the masked loop
#define MHQ_DEC_P3 0
#endif
#ifndef MHQ_DEC_LONG1  // 0: only the step before the end test resolves codes of 13+ bits
#define MHQ_DEC_LONG1 0
#endif
#ifndef MHQ_DEC_STEPS  // masked steps per end test of the probe loop (the plain decode)
#define MHQ_DEC_STEPS 3
#endif
#ifndef MHQ_DEC_LONGMID
#define MHQ_DEC_LONGMID 0
#endif
#ifndef MHQ_DEC_STEPS_GAPS  // the same for the in_end decode of framed strings (read_strings)
#define MHQ_DEC_STEPS_GAPS 2
#endif
#ifndef MHQ_DEC_NTLEN  // out_len / status as streaming stores (config 2 37.1 -> 35.7 us, config 3 32.9 -> 31.8)
#define MHQ_DEC_NTLEN 1
#endif
#ifndef MHQ_DEC_SOPEN  // 1: the first tile's input loads are addressed by two scalar loads (no wait for the offsets)
#define MHQ_DEC_SOPEN 0
#endif
#ifndef MHQ_DEC_OPTIMISTIC  // 1: literals whose region may truncate run the fast loop, checked after (see decode_piece)
#define MHQ_DEC_OPTIMISTIC 1
#endif
#ifndef MHQ_DEC_ENDOR  // 1: a literal's last output word is OR-ed in the end branch (0: by the next step)
#define MHQ_DEC_ENDOR 0
#endif
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
static_assert(kWOut % 16 == 0, "output slice must be whole 16-B chunks");

#ifndef MHQ_DEC_ALIGN  // a wave slice's alignment (16: its 16-B LDS accesses are single ds_*_b128)
#define MHQ_DEC_ALIGN 16
#endif
struct alignas(MHQ_DEC_ALIGN) WaveSmem {
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
__device__ void decode_literal_global(const uint8_t *src, uint64_t nbytes, uint8_t *dst, uint64_t cap,
                                      const Smem &sm, uint32_t *out_len, uint8_t *status) {
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
#if defined(MHQ_X_PLAINW)  // timing experiment only (wrong output)
    out_w[ow] = (uint32_t)acc;
#elif !defined(MHQ_X_NOOR)
    atomicOr(&out_w[ow], (uint32_t)acc);
#endif
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

// Ones at the bit positions >= d of a MSB-first word (d clamped to [0, 32]):
// the part of a staged word that lies at or past a literal's end.
__device__ __forceinline__ uint32_t ones_past(int32_t d) {
  const uint32_t c = (uint32_t)min(max(d, 0), 32);
  return (uint32_t)(0xffffffffull >> c);
}

// A literal's stream bits in registers with every bit past its end read as a
// one: `bb` holds bits [p, kb) MSB-aligned (zeros below); staged word kb/32
// (word index `wi`) is the next to enter; `left` = endbit - p and
// `rem` = endbit - kb, both signed.  With ones past the end the decode loop
// needs no end test: a well-formed literal ends in at most 7 padding ones, so
// the probe at the padding sees >= 30 ones (the EOS prefix) and stops there;
// a literal whose tail is not all ones decodes a code across its end, which
// `left < 0` shows (that literal is decoded again by the checked loop).
struct BitBufM {
  uint64_t bb;
  int32_t left, rem;
  uint32_t wi;
  const uint32_t *in_w;

  __device__ __forceinline__ void init(const uint32_t *words, uint32_t p0, uint32_t endbit) {
    in_w = words;
    const uint32_t k = p0 >> 5;
    const int32_t e = (int32_t)endbit - (int32_t)(32u * k);
    const uint32_t w0 = words[k] | ones_past(e), w1 = words[k + 1] | ones_past(e - 32);
    bb = (((uint64_t)w0 << 32) | w1) << (p0 & 31u);
    rem = e - 64;
    wi = k + 2u;
    left = (int32_t)(endbit - p0);
  }
  // The staged word that enters next (read early in a step, used by refill).
  __device__ __forceinline__ uint32_t next_word() const { return in_w[wi]; }
  // Tops the buffer up to >= 33 valid bits from `w` = next_word() when it
  // holds <= 32 (branch free).
  __device__ __forceinline__ void refill(uint32_t w) {
    const int32_t nb = left - rem;  // kb - p
    const bool need = nb <= 32;
    bb |= (uint64_t)(need ? (w | ones_past(rem)) : 0u) << ((uint32_t)(32 - nb) & 63u);
    rem -= need ? 32 : 0;
    wi += need ? 1u : 0u;
  }
  __device__ __forceinline__ uint32_t top32() const { return (uint32_t)(bb >> 32); }
  __device__ __forceinline__ void consume(uint32_t e) {
    bb <<= (e & 63u);
    left -= (int32_t)(e & 0xffu);
  }
};

// One step of the masked loop (>= 33 valid bits on entry).  The whole window
// is tested for the EOS prefix first (>= 30 ones: the literal ends here, see
// BitBufM); a first probe that meets a long code resolves it through LUT2
// with the whole window and skips the second probe (fewer than 12 valid bits
// may be left); otherwise two LUT1 probes.  LDS operations complete in issue
// order, so the previous step's output word (`pend`) and this step's refill
// word are issued after the first probe: the probe's wait does not include
// them.  The step's output word becomes the next `pend`, as 0 once a code has
// crossed the literal's end.  Returns true when the literal is finished:
// `stop` (EOS prefix at the step's start) or a crossing.
struct Pend {
  uint32_t ow, v;
};
// kLong false (the steps before the end test): a code of 13+ bits is left
// for the next step (its LUT1 entry is 0, so nothing is consumed: the step
// only refills), which saves the LUT2 branch in those steps.
template <bool kLong = true>
__device__ __forceinline__ bool masked_step(const Smem &sm, uint32_t *otgt, BitBufM &in, OutAcc &out, Pend &pend,
                                            bool &stop) {
  const uint32_t S = in.top32();
  stop = S >= 0xfffffffcu;
  uint32_t e = sm.lut1[S >> (32 - kLut1Bits)];
#if defined(MHQ_X_NOOR2)  // timing experiment only (wrong output): no OR, the word still computed
  asm volatile("" ::"v"(pend.v), "v"(pend.ow));
#elif !defined(MHQ_X_NOOR)
  atomicOr(&otgt[pend.ow], pend.v);
#endif
#ifdef MHQ_X_NOREFILL  // timing experiment only (wrong output): the refill word from registers, not LDS
  const uint32_t w = in.wi * 0x9e3779b9u;
#else
  const uint32_t w = in.next_word();
#endif
  bool lng = false;
  if (kLong && ((e == 0u) & !stop)) {  // a code of 13..29 bits (one branch: no short circuit)
    uint32_t sym = 0;
    const uint32_t L = long_code(sm.lut2, S, sym);
    e = L | (8u << 8) | (sym << 16);
    lng = true;
  }
  out.put(e >> 16, (e >> 8) & 0xffu);
  in.consume(e);
  uint32_t e2 = sm.lut1[in.top32() >> (32 - kLut1Bits)];
  e2 = lng ? 0u : e2;
  out.put(e2 >> 16, (e2 >> 8) & 0xffu);
  in.consume(e2);
#if MHQ_DEC_P3
  {
    // a third probe when its codes lie in the buffer's valid bits with two to
    // spare (the refill then tops up to >= 34) and its bytes fit the 64-bit
    // accumulator (one word leaves per step)
    uint32_t e3 = sm.lut1[in.top32() >> (32 - kLut1Bits)];
    const int32_t nb = in.left - in.rem;
    const bool take = (int32_t)(e3 & 0xffu) + 2 <= nb && out.ab + ((e3 >> 8) & 0xffu) <= 63u;
    e3 = take ? e3 : 0u;
    out.put(e3 >> 16, (e3 >> 8) & 0xffu);
    in.consume(e3);
  }
#endif
  in.refill(w);
  const bool ok = in.left >= 0;
  pend.ow = out.ow;
  pend.v = ok ? (uint32_t)out.acc : 0u;
  out.acc >>= out.ab & 32u;
  out.ow += out.ab >> 5;
  out.ab &= 31u;
  return stop || !ok;
}

#ifndef MHQ_DEC_LEAN  // 1: the lean fast loop (LDS pointers, no per-step crossing mask)
#define MHQ_DEC_LEAN 1
#endif
#ifndef MHQ_DEC_UNIFORM  // 1: the lean loop with wave-uniform control flow (branch-free move from A to B)
#define MHQ_DEC_UNIFORM 0
#endif
// The lean form of the fast loop's state: the output word and the next
// stream word are held as LDS pointers (their addresses need no arithmetic
// per step), and a step's output word is OR-ed whether or not a code crossed
// the literal's end -- a crossing makes the whole piece be decoded again by
// the checked loop over a re-zeroed output region (decode_piece), so stray
// bits of a malformed literal never survive.
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
struct BitBufL {  // BitBufM with the next word by pointer
  uint64_t bb;
  int32_t left, rem;
  const uint32_t *wp;
  __device__ __forceinline__ void init(const uint32_t *words, uint32_t p0, uint32_t endbit) {
    const uint32_t k = p0 >> 5;
    const int32_t e = (int32_t)endbit - (int32_t)(32u * k);
    const uint32_t w0 = words[k] | ones_past(e), w1 = words[k + 1] | ones_past(e - 32);
    bb = (((uint64_t)w0 << 32) | w1) << (p0 & 31u);
    rem = e - 64;
    wp = words + k + 2u;
    left = (int32_t)(endbit - p0);
  }
  __device__ __forceinline__ void refill(uint32_t w) {
    const int32_t nb = left - rem;  // kb - p
    const bool need = nb <= 32;
    bb |= (uint64_t)(need ? (w | ones_past(rem)) : 0u) << ((uint32_t)(32 - nb) & 63u);
    rem -= need ? 32 : 0;
    wp += need ? 1 : 0;
  }
  __device__ __forceinline__ uint32_t top32() const { return (uint32_t)(bb >> 32); }
  __device__ __forceinline__ void consume(uint32_t e) {
    bb <<= (e & 63u);
    left -= (int32_t)(e & 0xffu);
  }
};
struct PendL {
  uint32_t *p, v;
};
template <bool kLong = true>
__device__ __forceinline__ bool masked_step_lean(const Smem &sm, BitBufL &in, OutAccL &out, PendL &pend, bool &stop) {
  const uint32_t S = in.top32();
  stop = S >= 0xfffffffcu;
  uint32_t e = sm.lut1[S >> (32 - kLut1Bits)];
  atomicOr(pend.p, pend.v);
  const uint32_t w = *in.wp;
  bool lng = false;
  if (kLong && ((e == 0u) & !stop)) {  // a code of 13..29 bits (one branch: no short circuit)
    uint32_t sym = 0;
    const uint32_t L = long_code(sm.lut2, S, sym);
    e = L | (8u << 8) | (sym << 16);
    lng = true;
  }
  out.put(e >> 16, (e >> 8) & 0xffu);
  in.consume(e);
  uint32_t e2 = sm.lut1[in.top32() >> (32 - kLut1Bits)];
  e2 = lng ? 0u : e2;
  out.put(e2 >> 16, (e2 >> 8) & 0xffu);
  in.consume(e2);
  in.refill(w);
  pend.p = out.op;
  pend.v = (uint32_t)out.acc;
  const uint32_t t = out.ab & 32u;
  out.acc >>= t;
  out.op += t >> 5;
  out.ab &= 31u;
  return stop || in.left < 0;
}

#ifndef MHQ_DEC_WIN  // 1: the lean loop reads each step's 64-bit window afresh (no refill state); 3: its top 32 bits by v_alignbit
#define MHQ_DEC_WIN 3
#endif
// A literal's stream with no refill state: each step reads the two staged
// words holding bit p (one ds_read2) and shifts them to a window of >= 33
// valid bits, bits past the literal's end forced to ones (so the stop and
// crossing rules are those of BitBufM).  Fewer instructions per step than the
// refill; the window read is one more LDS round trip on the step's chain.
struct WinBuf {
  uint32_t pa;    // bit position as an LDS bit address: 8 * (byte address of the staged words) + p
  int32_t left;   // endbit - p
  __device__ __forceinline__ void init(const uint32_t *words, uint32_t p0, uint32_t endbit) {
    pa = 8u * (uint32_t)(uintptr_t)words + p0;
    left = (int32_t)(endbit - p0);
  }
  __device__ __forceinline__ uint64_t window() const {
    typedef __attribute__((address_space(3))) const uint32_t lds_u32;
    lds_u32 *w = (lds_u32 *)(uintptr_t)((pa >> 3) & ~3u);
    const uint64_t x = ((uint64_t)w[0] << 32) | w[1];
    // ones from bit `left` (MSB first) on, in the high word only: the probes
    // and the stop test read the top 32 bits, and a second probe's 12 bits
    // lie in them too (the first consumes at most 12)
    const uint32_t c = (uint32_t)min(max(left, 0), 32);
    return (x << (pa & 31u)) | ((uint64_t)(uint32_t)(0xffffffffull >> c) << 32);
  }
};
// MHQ_DEC_WIN 3: the window as its top 32 bits only, one v_alignbit of the
// two staged words (no 64-bit shift, no word swap).  The state is the bit
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

template <bool kLong = true>
__device__ __forceinline__ bool win_step32(const Smem &sm, WinBuf3 &in, OutAccL &out, PendL &pend, bool &stop) {
  const uint32_t S = in.top();
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
  const uint32_t t = out.ab & 32u;
  out.acc >>= t;
  out.op += t >> 5;
  out.ab &= 31u;
  return stop || in.left < 0;
}

template <bool kLong = true, class WB>
__device__ __forceinline__ bool win_step(const Smem &sm, const uint32_t *words, WB &in, OutAccL &out,
                                         PendL &pend, bool &stop) {
  const uint64_t W = in.window();
  const uint32_t S = (uint32_t)(W >> 32);
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
  const uint64_t W2 = W << (e & 63u);
  uint32_t e2 = sm.lut1[(uint32_t)(W2 >> 32) >> (32 - kLut1Bits)];
  e2 = lng ? 0u : e2;
  out.put(e2 >> 16, (e2 >> 8) & 0xffu);
  const uint32_t n = (e & 0xffu) + (e2 & 0xffu);
  in.pa += n;
  in.left -= (int32_t)n;
  pend.p = out.op;
  pend.v = (uint32_t)out.acc;
  const uint32_t t = out.ab & 32u;
  out.acc >>= t;
  out.op += t >> 5;
  out.ab &= 31u;
  return stop || in.left < 0;
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
  __device__ __forceinline__ uint32_t rd(const uint32_t *q, uint32_t k) const { return __builtin_bswap32(q[k ^ swz]); }
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
__device__ __noinline__ uint32_t decode_checked(const Smem &sm, WaveSmem &ws, uint32_t p, uint32_t endbit,
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
    out.flush(ws.out_w);
  }
  const uint32_t oend_got = out.optr();
  bad = oend_got != oend ? bad : 0u;
  return (oend_got - ostart) | (bad << 31);
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

#ifdef MHQ_DIAG_COUNT
__device__ unsigned long long g_cnt[8];
#endif
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
template <bool kGaps>
__device__ __forceinline__ void load_off(TileOff &t, const uint64_t *__restrict__ in_off,
                                         const uint32_t *__restrict__ in_end, const uint64_t *__restrict__ out_off,
                                         uint64_t s, uint64_t L1, uint32_t tl, uint32_t lane) {
  const uint32_t z = vzero();  // keeps the loads per-lane vector loads
  const uint64_t j0 = min(s + 2u * lane, L1) + z, j1 = min(s + 2u * lane + 1u, L1) + z;
  const uint64_t je = min(s + (uint64_t)tl, L1) + z;
  t.i0 = in_off[j0];
  t.i1 = lo32(in_off, j1);
  if (kGaps) {  // (in_end has n entries: indices clamped below L1)
    t.e0 = in_end[min(j0, L1 - 1u)];
    t.e1 = in_end[min(j1, L1 - 1u)];
  }
  t.o0 = out_off[j0];
  t.o1 = lo32(out_off, j1);
  t.ie = in_off[je];
  t.oe = out_off[je];
}

// The two halves of load_off, for the launch's opening.
template <bool kGaps>
__device__ __forceinline__ void load_off_in(TileOff &t, const uint64_t *__restrict__ in_off,
                                            const uint32_t *__restrict__ in_end, uint64_t s, uint64_t L1,
                                            uint32_t tl, uint32_t lane) {
  const uint32_t z = vzero();
  const uint64_t j0 = min(s + 2u * lane, L1) + z, j1 = min(s + 2u * lane + 1u, L1) + z;
  const uint64_t je = min(s + (uint64_t)tl, L1) + z;
  t.i0 = in_off[j0];
  t.i1 = lo32(in_off, j1);
  if (kGaps) {
    t.e0 = in_end[min(j0, L1 - 1u)];
    t.e1 = in_end[min(j1, L1 - 1u)];
  }
  t.ie = in_off[je];
}
__device__ __forceinline__ void load_off_out(TileOff &t, const uint64_t *__restrict__ out_off, uint64_t s,
                                             uint64_t L1, uint32_t tl, uint32_t lane) {
  const uint32_t z = vzero();
  const uint64_t j0 = min(s + 2u * lane, L1) + z, j1 = min(s + 2u * lane + 1u, L1) + z;
  const uint64_t je = min(s + (uint64_t)tl, L1) + z;
  t.o0 = out_off[j0];
  t.o1 = lo32(out_off, j1);
  t.oe = out_off[je];
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

// out_len / status of literals [s, s + m) from the wave's len array.
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
#if MHQ_DEC_NTLEN
      __builtin_nontemporal_store(len, out_len + s + j);
      __builtin_nontemporal_store((uint8_t)st, status + s + j);
#else
      out_len[s + j] = len;
      status[s + j] = (uint8_t)st;
#endif
    }
  }
}

// Decodes the m literals whose boundary records rec[0..m] and input bytes are
// staged: zero the output region, sort, decode into out_w / len.
#ifndef MHQ_DEC_LOOPPRIO  // probe-loop priority by the wave's tile count (0: all loops at priority 0)
#define MHQ_DEC_LOOPPRIO 2
#endif
// A wave's loop priority: with every loop at one priority the SIMD issues
// oldest-first, so a SIMD's three waves finish their equal work one after the
// other and the last runs alone (the age staircase).  Loops of
// earlier tiles at a higher priority let the younger waves catch up at every
// tile boundary.
[[maybe_unused]] __device__ __forceinline__ void set_loop_prio(uint32_t p) {
  if (p >= 2u)
    __builtin_amdgcn_s_setprio(2);
  else if (p == 1u)
    __builtin_amdgcn_s_setprio(1);
  else
    __builtin_amdgcn_s_setprio(0);
}

template <bool kGaps>
__device__ __forceinline__ void decode_piece(const Smem &sm, WaveSmem &ws, uint32_t m, uint32_t out_bytes,
                                             uint32_t lane, [[maybe_unused]] int tls = -1, uint32_t prio = 0) {
  // masked steps per end test: 3 for the plain decode (north star -2.7 %,
  // config 4 -7 %, print +3 %: profiles/r04c_decode_steps_ab.txt); the read
  // path keeps 2 (one unexplained fault of a read test with 3)
  constexpr int kSteps = kGaps ? MHQ_DEC_STEPS_GAPS : MHQ_DEC_STEPS;
  for (uint32_t c = lane; c < (out_bytes + 15u) >> 4; c += kWave) *(u32x4 *)(ws.out_w + 4u * c) = u32x4{0u, 0u, 0u, 0u};
#ifdef MHQ_X_DBLZERO  // timing experiment: the zeroing twice
  wave_sync();
  for (uint32_t c = lane; c < (out_bytes + 15u) >> 4; c += kWave) *(u32x4 *)(ws.out_w + 4u * c) = u32x4{0u, 0u, 0u, 0u};
#endif
#ifdef MHQ_X_DBLSORT  // timing experiment: the sort twice
  for (int rep = 0; rep < 2; rep++)
#endif
  {
#ifdef MHQ_X_NOSORT  // timing experiment only: literals in tile order, lane t on t and 127 - t
  if (lane < m) ws.order[lane] = (uint8_t)lane;
  if (lane + kWave < m) ws.order[lane + kWave] = (uint8_t)(lane + kWave);
  wave_sync();
#else
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
#endif
  }
  // Lane t decodes rank t, then rank 127 - t if there is one: the 64 longest
  // literals one per lane, the rest on the lanes with the shortest of those
  // (LPT).  The lane's two fast loops run back to back in one loop (it moves
  // to its second literal in place), so lanes stay busy until all are done;
  // the short checked tails follow, one literal at a time.
#ifdef MHQ_X_NODEC  // timing experiment only: sort and zero, no decode
  if (lane < m) ws.len[lane] = 0;
  wave_sync();
  return;
#endif
  const bool hasA = lane < m, hasB = 2u * kWave - 1u - lane < m;
  LitRef<kGaps> A, B;
  A.load(ws, hasA ? ws.order[lane] : 0u);
  B.load(ws, hasB ? ws.order[2u * kWave - 1u - lane] : 0u);
  const uint32_t ostartA = A.optr, ostartB = B.optr;
  TL(tls);
#if MHQ_DEC_LOOPPRIO
  set_loop_prio(prio);
#elif MHQ_DEC_PRIO
  __builtin_amdgcn_s_setprio(0);  // the probe loop at normal priority
#endif
  // Every literal runs the masked loop to its end (ones past the end: no end
  // test, no separate tail loop); the lane moves from A to B in place.  A
  // literal with a code across its end (not well formed) takes the checked
  // loop.  So does, since round 3, a piece in which a literal whose region
  // can truncate (under floor(8 bits / 5) bytes) turned out not to fit it
  // (below): regions sized to the exact plaintext -- a caller that knows the
  // lengths, as every round trip does -- stay on the fast loop.
  constexpr uint32_t kRedo = 0xffffffffu;
  const bool roomA = hasA && (A.roomy() || (MHQ_DEC_OPTIMISTIC && A.in_slice()));
  const bool roomB = hasB && (B.roomy() || (MHQ_DEC_OPTIMISTIC && B.in_slice()));
  uint32_t rA = kRedo, rB = kRedo;
#if MHQ_DEC_LEAN
#if MHQ_DEC_UNIFORM
  {
    // Wave-uniform control flow: the loop runs while any lane has a literal
    // left, and the move from A to B is branch free.  A lane with nothing
    // left is frozen on an all-ones window: every step stops at once,
    // consumes nothing and ORs its last word again (idempotent), and its
    // result is recomputed unchanged.
    BitBufL in, inB;  // inB: B's stream, set up once for the in-loop switch
    in.init(ws.in_w, roomA ? A.p : B.p, roomA ? A.endbit : B.endbit);
    inB.init(ws.in_w, B.p, B.endbit);
    OutAccL out, outB;
    out.init(ws.out_w, roomA ? A.optr : B.optr);
    outB.init(ws.out_w, B.optr);
    uint32_t ost = roomA ? ostartA : ostartB;
    PendL pend{out.op, 0u};
    bool onB = !roomA, active = roomA || roomB;
    if (!active) in.bb = ~0ull;
    while (__ballot(active)) {
      bool stop;
#pragma unroll
      for (int k = 1; k < kSteps; k++) masked_step_lean<MHQ_DEC_LONG1 != 0>(sm, in, out, pend, stop);
      const bool fin = masked_step_lean(sm, in, out, pend, stop);
      // stop: the EOS prefix (INVALID when a 31st bit of the literal follows);
      // left < 0: a code crossed the end (the piece is redone, below)
      const uint32_t r = in.left < 0 ? kRedo : (out.optr(ws.out_w) - ost) | ((uint32_t)(in.left > kEosOnes) << 31);
      rA = fin && !onB ? r : rA;
      rB = fin && onB ? r : rB;
      const bool sw = fin && !onB && roomB;  // A done: on to B
      active = active && (!fin || sw);
      in.bb = sw ? inB.bb : (active ? in.bb : ~0ull);
      in.left = sw ? inB.left : in.left;
      in.rem = sw ? inB.rem : in.rem;
      in.wp = sw ? inB.wp : in.wp;
      out.acc = sw ? 0ull : out.acc;
      out.op = sw ? outB.op : out.op;
      out.ab = sw ? outB.ab : out.ab;
      ost = sw ? ostartB : ost;
      onB = onB || sw;
    }
    atomicOr(pend.p, pend.v);
  }
#elif MHQ_DEC_WIN
  {
#if MHQ_DEC_WIN == 3
    WinBuf3 in;
#define MHQ_WSTEP(K) win_step32<K>(sm, in, out, pend, stop)
#else
    WinBuf in;
#define MHQ_WSTEP(K) win_step<K>(sm, ws.in_w, in, out, pend, stop)
#endif
    in.init(ws.in_w, roomA ? A.p : B.p, roomA ? A.endbit : B.endbit);
    OutAccL out;
    out.init(ws.out_w, roomA ? A.optr : B.optr);
    uint32_t ost = roomA ? ostartA : ostartB;
    PendL pend{out.op, 0u};
    bool onB = !roomA, active = roomA || roomB;
    while (active) {
      bool stop;
#if MHQ_DEC_LONGMID  // experiment: the steps after the first resolve long codes too
      MHQ_WSTEP(MHQ_DEC_LONG1 != 0);
#pragma unroll
      for (int k = 2; k < kSteps; k++) MHQ_WSTEP(true);
#else
#pragma unroll
      for (int k = 1; k < kSteps; k++) MHQ_WSTEP(MHQ_DEC_LONG1 != 0);
#endif
      if (MHQ_WSTEP(true)) {
        const uint32_t r = in.left < 0 ? kRedo : (out.optr(ws.out_w) - ost) | ((uint32_t)(in.left > kEosOnes) << 31);
        rA = onB ? rA : r;
        rB = onB ? r : rB;
        active = !onB && roomB;
        in.init(ws.in_w, B.p, B.endbit);
        out.init(ws.out_w, B.optr);
        ost = ostartB;
        onB = true;
      }
    }
    atomicOr(pend.p, pend.v);
#undef MHQ_WSTEP
  }
#else
  {
    BitBufL in, inB;  // inB: B's stream, set up once for the in-loop switch
    in.init(ws.in_w, roomA ? A.p : B.p, roomA ? A.endbit : B.endbit);
    inB.init(ws.in_w, B.p, B.endbit);
    OutAccL out;
    out.init(ws.out_w, roomA ? A.optr : B.optr);
    uint32_t ost = roomA ? ostartA : ostartB;
    PendL pend{out.op, 0u};
    bool onB = !roomA, active = roomA || roomB;
    while (active) {
      bool stop;
#pragma unroll
      for (int k = 1; k < kSteps; k++) masked_step_lean<MHQ_DEC_LONG1 != 0>(sm, in, out, pend, stop);
      if (masked_step_lean(sm, in, out, pend, stop)) {
        // stop: the EOS prefix (INVALID when a 31st bit of the literal follows);
        // left < 0: a code crossed the end (the piece is redone, below)
        const uint32_t r = in.left < 0 ? kRedo : (out.optr(ws.out_w) - ost) | ((uint32_t)(in.left > kEosOnes) << 31);
        rA = onB ? rA : r;
        rB = onB ? r : rB;
        active = !onB && roomB;
        in = inB;  // (unused unless active)
        out.init(ws.out_w, B.optr);
        ost = ostartB;
        onB = true;
      }
    }
    atomicOr(pend.p, pend.v);
  }
#endif
  // a lane that ran a literal through the fast loop and got no result crossed its end
  const bool crossed = (roomA && rA == kRedo) || (roomB && rB == kRedo);
#else
  constexpr bool crossed = false;
  {
    BitBufM in, inB;  // inB: B's stream, set up once for the in-loop switch
    in.init(ws.in_w, roomA ? A.p : B.p, roomA ? A.endbit : B.endbit);
    inB.init(ws.in_w, B.p, B.endbit);
    OutAcc out;
    out.init(roomA ? A.optr : B.optr);
    uint32_t ost = roomA ? ostartA : ostartB;
    Pend pend{out.ow, 0u};
    bool onB = !roomA, active = roomA || roomB;
    while (active) {
#ifdef MHQ_DIAG_COUNT
      {
        const uint64_t mask = __ballot(1);
        if (lane == (uint32_t)__builtin_ctzll(mask)) {
          atomicAdd(&g_cnt[0], 1ull);
          atomicAdd(&g_cnt[1], (unsigned long long)__popcll(mask));
        }
      }
#endif
      bool stop;
      // MHQ_DEC_STEPS steps per end test: a finished literal (EOS prefix, or
      // a code across its end) stays finished through further steps (no bits
      // consumed at the EOS prefix; `left` stays negative, the word held
      // back), so the last step's result covers them all
#pragma unroll
      for (int k = 1; k < kSteps; k++) masked_step<MHQ_DEC_LONG1 != 0>(sm, ws.out_w, in, out, pend, stop);
      if (masked_step(sm, ws.out_w, in, out, pend, stop)) {
        // stop: the EOS prefix at p (INVALID when a 31st bit of the literal follows)
        const uint32_t r = in.left < 0 ? kRedo : (out.optr() - ost) | ((uint32_t)(in.left > kEosOnes) << 31);
#if MHQ_DEC_ENDOR
        atomicOr(&ws.out_w[pend.ow], pend.v);  // the literal's last word
        pend.v = 0u;
#endif
        // (otherwise the literal's last word stays in `pend`: the next step
        // ORs it before anything else, as every step does its predecessor's,
        // and the loop's end ORs the last one -- no extra LDS store here)
        rA = onB ? rA : r;
        rB = onB ? r : rB;
        active = !onB && roomB;
        in = inB;  // (unused unless active)
        out.init(B.optr);
        ost = ostartB;
        onB = true;
      }
    }
#if !MHQ_DEC_ENDOR
    atomicOr(&ws.out_w[pend.ow], pend.v);
#endif
  }
#endif
#if MHQ_DEC_OPTIMISTIC || MHQ_DEC_LEAN
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
    const bool badA = hasA && MHQ_DEC_OPTIMISTIC && overflow(A, rA);
    const bool badB = hasB && MHQ_DEC_OPTIMISTIC && overflow(B, rB);
    if (__ballot(badA || badB || crossed)) {
      wave_sync();
      for (uint32_t c = lane; c < (out_bytes + 15u) >> 4; c += kWave) *(u32x4 *)(ws.out_w + 4u * c) = u32x4{0u, 0u, 0u, 0u};
      wave_sync();
      rA = kRedo;
      rB = kRedo;
    }
  }
#endif
  TL(tls < 0 ? -1 : tls + 1);
  if (hasA) ws.len[A.lit] = rA != kRedo ? rA : decode_checked(sm, ws, A.p, A.endbit, A.optr, A.oend);
  if (hasB) ws.len[B.lit] = rB != kRedo ? rB : decode_checked(sm, ws, B.p, B.endbit, B.optr, B.oend);
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
struct OutAccG {
  uint64_t acc;
  uint32_t ow, ab, owf, first, rs, ga, q0, q1, q2, q3;
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
#ifndef MHQ_X_LONG_NOSTORE  // timing experiment only: no output stores from the long path
    if (full && ow >= owf) {
      if (!grouped(ow)) {
        gout[ow] = v;
      } else {
        const uint32_t r = (ow + ga) & 3u;
        q0 = r == 0u ? v : q0;
        q1 = r == 1u ? v : q1;
        q2 = r == 2u ? v : q2;
        q3 = r == 3u ? v : q3;
        if (r == 3u) *(u32x4 *)(gout + ow - 3u) = u32x4{q0, q1, q2, v};
      }
    }
#endif
    first = (full && ow < owf) ? v : first;
    acc >>= ab & 32u;
    ow += ab >> 5;
    ab &= 31u;
  }
  __device__ __forceinline__ void finish(uint32_t *gout) {
    flush(gout);
    // whole words of the last, incomplete 16-B group
    if (grouped(ow)) {
      const uint32_t r = (ow + ga) & 3u, g = ow - r;
      if (r > 0u) gout[g] = q0;
      if (r > 1u) gout[g + 1u] = q1;
      if (r > 2u) gout[g + 2u] = q2;
    }
    uint8_t *g8 = (uint8_t *)gout;
    const uint32_t hi = ab >> 3, lo = ow < owf ? (rs & 3u) : 0u;
    if (ow >= owf && (rs & 3u)) {
      for (uint32_t x = rs & 3u; x < 4u; x++) g8[(owf - 1u) * 4u + x] = (uint8_t)(first >> (8u * x));
    }
    for (uint32_t x = lo; x < hi; x++) g8[ow * 4u + x] = (uint8_t)(acc >> (8u * x));
  }
  __device__ __forceinline__ uint32_t optr() const { return ow * 4u + (ab >> 3); }
};

// The checked loop of decode_checked on a window, with the lane's running
// accumulator (roomy literals only: no buffer-full rule).  Returns the status.
template <class BB>
__device__ __forceinline__ uint32_t end_checked_g(const Smem &sm, const uint32_t *win, uint32_t p, uint32_t endbit,
                                                  OutAccG &out, uint32_t *gout, uint32_t swz) {
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
template <class Acc, class BB, bool kFlush = true>
__device__ __forceinline__ void long_step(const Smem &sm, uint32_t *otgt, BB &in, Acc &out, uint32_t endbit,
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

template <bool kGaps>
__device__ void decode_tile_long(const Smem &sm, WaveSmem &ws, const uint8_t *__restrict__ in,
                                 const uint64_t *__restrict__ in_off, const uint32_t *__restrict__ in_end,
                                 uint64_t in_bias, uint8_t *__restrict__ out,
                                 const uint64_t *__restrict__ out_off, uint64_t out_bias,
                                 uint32_t *__restrict__ out_len, uint8_t *__restrict__ status, uint64_t s,
                                 uint32_t cnt, uint32_t lane, const uint8_t *__restrict__ str_kind = nullptr) {
  uint32_t *win = ws.in_w + lane * kLongWords;  // spans the input and output slices
  const uint32_t swz = (lane & 7u) << 2;         // BitBufS: the window's chunk swizzle
  constexpr uint32_t kWinBits = kLongWords * 32u;
  constexpr uint32_t kSafe = kWinBits - 96u;  // fast steps stay below: 24 bits + two words of look-ahead
  uint32_t j = lane;
  bool have = false;
  uint64_t ib = 0, ie = 0, ob = 0;
  uint64_t rel = 0;  // bits of the literal consumed
  uint32_t *gout = nullptr;
  OutAccG acc;
  acc.init(0);
  uint32_t ostart = 0;
  // next literal of this lane (roomy ones stay; the rest are done at once from global memory)
  auto next_lit = [&]() {
    have = false;
    while (j < cnt) {
      ib = in_off[s + j];
      if (kGaps) {  // the end's low word: the end is the first at or after ib with it
        const uint32_t e = in_end[s + j];
        ie = (ib & ~0xffffffffull) | e;
        if (e < (uint32_t)ib) ie += 1ull << 32;
      } else {
        ie = in_off[s + j + 1];
      }
      ob = out_off[s + j];
      const uint64_t oe = out_off[s + j + 1];
      uint8_t *o = out + (ob - out_bias);
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
        rel = 0;
        have = true;
        return;
      }
      j += kWave;
    }
  };
  next_lit();
#ifdef MHQ_X_LONG_NOSTAGE
  bool staged_once = false;
#endif
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
      nck = min((uint32_t)(((uintptr_t)last - (uintptr_t)a16) >> 4) + 1u, kLongWords / 4u);
      p = delta * 8u + (uint32_t)(rel & 7u);
      endw = p + (uint32_t)((ie - ib) * 8u - rel);  // the literal's end in window bits (may lie beyond)
    }
#ifdef MHQ_X_LONG_NOSTAGE  // timing experiment only (wrong output): windows staged in the first round only
    if (!staged_once)
#endif
#pragma unroll
    for (uint32_t k = 0; k < kWave / 8u; k++) {
      // slot lane % 8 of owner o's window takes chunk (lane % 8) ^ (o % 8)
      const uint32_t o = 8u * k + (lane >> 3), c = (lane & 7u) ^ (lane >> 3);
      const uint64_t so = (uint64_t)__shfl((unsigned long long)src, (int)o);
      const uint32_t no = (uint32_t)__shfl((int)nck, (int)o);
      if (c < no)  // chunks past the literal's last one stay unloaded: their bits are never consumed
        __builtin_amdgcn_global_load_lds((g_void *)(uintptr_t)(so + 16u * c), (lds_void *)(ws.in_w + 256u * k), 16, 0,
                                         0);
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
#ifdef MHQ_X_LONG_NOSTAGE
    staged_once = true;
#endif
    wave_sync();
    if (have) {
      const bool ends_here = endw + 64u <= kWinBits;
      BitBufS bin;
      bin.init(win, p, swz);
      uint32_t bad = 0;
      const int lim0 = ends_here ? (int)endw - 24 : (int)kSafe;
      int lim = lim0;
#ifdef MHQ_X_LONG_NODEC  // timing experiment only: windows staged, nothing decoded
      if ((int)bin.p <= lim) bin.p = (uint32_t)lim + 1u;
#else
      // two probes per flush while two codes (<= 30 bits each) surely fit,
      // then single ones up to the end test's bound
      const int lim2 = lim0 - 30;
      while ((int)bin.p <= lim2 && lim != -1) {
        long_step<OutAccG, BitBufS, false>(sm, gout, bin, acc, endw, lim, bad);
        if (lim != -1) long_step<OutAccG, BitBufS, false>(sm, gout, bin, acc, endw, lim, bad);
        acc.flush(gout);
      }
      while ((int)bin.p <= lim) long_step(sm, gout, bin, acc, endw, lim, bad);
#endif
      const bool stopped = lim == -1 && lim0 != -1;  // a fast step finished the literal (EOS prefix, long code past the end)
      if (stopped || ends_here) {
        const uint32_t st = stopped ? bad : end_checked_g<BitBufS>(sm, win, bin.p, endw, acc, gout, swz);
        uint32_t got = acc.optr() - ostart, st2 = st;
        acc.finish(gout);
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

// Slow path: a tile whose bytes exceed the slices, in greedy pieces staged
// synchronously from global memory; a literal larger than a slice alone is
// decoded by lane 0 from global memory.
__device__ void decode_tile_pieces(const Smem &sm, WaveSmem &ws, const uint8_t *__restrict__ in,
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
    store_out(oa - odelta, (const uint8_t *)ws.out_w, odelta, out_bytes, lane);
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
  const uint64_t fin_gate = kGaps && str.finish_needed ? __builtin_nontemporal_load(str.finish_needed) : 0;
#if MHQ_DEC_SOPEN
  // The first tile's input range comes from two scalar loads (the tile's first
  // and one-past-last literal), so its input loads are issued without waiting
  // for the per-lane offsets, which load alongside.
  const uint64_t s0 = L0 + (uint64_t)__builtin_amdgcn_readfirstlane(tile) * tl0;
  const uint64_t ib0 = in_off[min(s0, L1)], ie0 = in_off[min(s0 + (uint64_t)tl0, L1)];
  TileIn tin;
  uint32_t keep[kPF] = {};
  load_in(tin, in, in_bias, ib0, ie0, lane, keep);
  load_off_in<kGaps>(off, in_off, in_end, L0 + (uint64_t)tile * tl0, L1, tl0, lane);
#else
  load_off_in<kGaps>(off, in_off, in_end, L0 + (uint64_t)tile * tl0, L1, tl0, lane);
  TileIn tin;
  uint32_t keep[kPF] = {};
  load_in(tin, in, in_bias, uniform64(off.i0), uniform64(off.ie), lane, keep);
#endif
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
#if MHQ_DEC_PRIO
    __builtin_amdgcn_s_setprio(MHQ_DEC_PRIO);  // staging, flush and sort (serial phases) ahead of other waves' loops
#endif
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
#ifdef MHQ_X_DBLSTAGE  // timing experiment: the staging writes twice
      wave_sync();
#pragma unroll
      for (int k = 0; k < kPF; k++) {
        const uint32_t c = lane + (uint32_t)kWave * k;
        if (c < chunks) put_chunk(ws, c, tin.v[k]);
      }
#endif
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
      store_out(pd_o, (const uint8_t *)ws.out_w, pd_lo, pd_hi, lane);
#ifdef MHQ_X_DBLFLUSH  // timing experiment: the output flush twice
      wave_sync();
      store_out(pd_o, (const uint8_t *)ws.out_w, pd_lo, pd_hi, lane);
#endif
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
#if MHQ_DEC_LOOPPRIO == 2
      decode_piece<kGaps>(sm, ws, cnt, out_bytes, lane, tl_slot(tl_j, 3), tl_j < 2u ? 1u : 0u);
#else
      decode_piece<kGaps>(sm, ws, cnt, out_bytes, lane, tl_slot(tl_j, 3), tl_j < 2u ? 2u - tl_j : 0u);
#endif
      pd_o = oa - odelta;
      pd_lo = odelta;
      pd_hi = out_bytes;
      pd_s = s;
      pd_m = cnt;
    } else {
      // a tile a little over the slice (short literals with a few long ones)
      // goes in staged pieces; one of long literals streams through windows
      // (kGaps: every such tile streams)
#ifdef MHQ_X_NOLONG  // timing experiment: the piece path for every oversized tile
      if (!kGaps)
#else
      if (!kGaps && (ie - ib) <= 2u * (uint64_t)kWIn && (oe - ob) <= 2u * (uint64_t)kWOut)
#endif
        decode_tile_pieces(sm, ws, in, in_off, in_bias, out, out_off, out_bias, out_len, status, s, cnt, lane);
      else
        decode_tile_long<kGaps>(sm, ws, in, in_off, in_end, in_bias, out, out_off, out_bias, out_len, status, s,
                                cnt, lane, kGaps ? str.kind : nullptr);
    }
    TL(tl_slot(tl_j, 5));
    tl_j++;
    tile = tile2;
    tile2 = tile3;
    tile3 = __builtin_amdgcn_readfirstlane(tile4);
  }
  if (pd_o) {
    store_out(pd_o, (const uint8_t *)ws.out_w, pd_lo, pd_hi, lane);
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
            copy_bytes(out + (o0 - out_bias), str.blk + st0, take);
            out_len[i] = (uint32_t)take;
          }
        }
      }
    }
  }
  TL(63);
}

template <bool kGaps>
__global__ __launch_bounds__(kT) void decode_kernel(const uint8_t *__restrict__ in, const uint64_t *__restrict__ in_off,
                                                    const uint32_t *__restrict__ in_end, StrFinish str,
                                                    uint64_t in_bias, uint64_t n, uint8_t *__restrict__ out,
                                                    const uint64_t *__restrict__ out_off, uint64_t out_bias,
                                                    uint32_t *__restrict__ out_len, uint8_t *__restrict__ status,
                                                    const uint32_t *__restrict__ g_lut1,
                                                    const uint16_t *__restrict__ g_lut2,
                                                    const uint8_t *__restrict__ g_len, uint64_t per_block,
                                                    uint32_t tl0) {
  __shared__ Smem sm;
  decode_body<kGaps>(sm, in, in_off, in_end, str, in_bias, n, out, out_off, out_bias, out_len, status, g_lut1, g_lut2,
                     g_len, per_block, tl0);
}

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
};

struct RsTile {  // pos / limit / prefix of strings s + 2 lane + {0, 1}; pos of string s + tile
  uint64_t p0, p1, l0, l1, pe;
  uint32_t pf;  // prefix of the first | of the second << 8
};

__device__ __forceinline__ void rs_load(RsTile &t, const RsArgs &a, uint64_t s, uint64_t L1, uint32_t tl,
                                        uint32_t lane) {
  const uint32_t z = vzero();
  const uint64_t j0 = min(s + 2u * lane, L1 - 1u) + z, j1 = min(s + 2u * lane + 1u, L1 - 1u) + z;
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
#if MHQ_DEC_NTLEN
      __builtin_nontemporal_store(len, out_len + s + j);
      __builtin_nontemporal_store((uint8_t)st, status + s + j);
#else
      out_len[s + j] = len;
      status[s + j] = (uint8_t)st;
#endif
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
#if MHQ_DEC_PRIO
    __builtin_amdgcn_s_setprio(MHQ_DEC_PRIO);
#endif
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
      store_out(pd_o, (const uint8_t *)ws.out_w, pd_lo, pd_hi, lane);
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
          return fits ? slice_byte(ws, (uint32_t)(q - ps) + idelta) : (uint32_t)a.blk[q];
        });
        if (r.far)  // a header octet outside the staged span: from global memory (bad below unless it failed)
          r = rs_parse(p, lim, pf, blk_len, 0, blk_len, [&](uint64_t q) -> uint32_t { return a.blk[q]; });
        bad |= r.start + r.take > min(pn, blk_len);  // read_parse_kernel's order test
        const uint32_t k = r.kind & 3u;
        const uint64_t hend = k == 1u ? r.start + r.take : r.start;
        const uint64_t reg = region_at(r.start), i = s + j;
        kinds |= r.kind << (4 * h);
        if (k == 0u) (h ? raw1 : raw0) = (uint32_t)r.take;
        a.out_off[i] = reg;  // (streaming stores: 1.6 us slower)
        a.next[i] = k == 2u ? p : r.start + r.take;
        if (fits) {
          ws.rec[j] = (uint32_t)(r.start - ps + idelta) | (uint32_t)(reg - rs0 + odelta) << 16;
          ws.len[j] = (uint32_t)(hend - ps + idelta);
        } else {
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
      decode_piece<true>(sm, ws, cnt, out_bytes, lane, -1, tl_j < 2u ? 1u : 0u);
      // raw payloads into their regions
#pragma unroll
      for (int h = 0; h < 2; h++) {
        const uint32_t j = 2u * lane + (uint32_t)h, take = h ? raw1 : raw0;
        if (j < cnt && ((kinds >> (4 * h)) & 3u) == 0u) {
          const uint32_t r = ws.rec[j], x = r & 0xffffu, y = r >> 16;
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
      if (lane == 0 && s + cnt < a.n) {
        const uint64_t i = s + cnt;
        const RsStr r = rs_parse(a.pos[i], min(a.limit[i], blk_len), a.prefix[i], blk_len, 0, blk_len,
                                 [&](uint64_t q) -> uint32_t { return a.blk[q]; });
        a.out_off[i] = region_at(r.start);
      }
      __threadfence_block();
      wave_sync();
      decode_tile_long<true>(sm, ws, a.blk, a.sc_start, a.sc_hend, 0, a.out, a.out_off, 0, a.out_len, a.status, s,
                             cnt, lane, a.sc_kind);
      __threadfence_block();
      for (uint32_t j = lane; j < cnt; j += kWave) {  // the lane that wrote string j's length
        const uint64_t i = s + j;
        const uint8_t kd = a.sc_kind[i];
        if ((kd & 3u) != 0u) continue;
        const uint64_t st0 = a.sc_start[i], take = a.next[i] - st0;
        if (take) {
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
    store_out(pd_o, (const uint8_t *)ws.out_w, pd_lo, pd_hi, lane);
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
  uint64_t *wg_agg;  // per workgroup: gen's low 24 bits << 40 | capacity sum
  uint64_t *wg_fin;  // per workgroup: gen when its range holds a raw string
};
constexpr uint64_t kAggBits = 40;  // a workgroup's capacity sum < 2^40

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
  const uint64_t tag = (a.gen & 0xffffffull) << kAggBits;
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
      for (;;) {
        v = __hip_atomic_load((unsigned long long *)f.wg_agg + g, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        if ((v & ~((1ull << kAggBits) - 1u)) == tag) break;
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

#ifdef MHQ_DIAG_COUNT
extern "C" int mhq_diag_read(unsigned long long *out, int n) {
  unsigned long long h[8];
  if (hipMemcpyFromSymbol(h, HIP_SYMBOL(g_cnt), sizeof(h)) != hipSuccess) return -1;
  for (int i = 0; i < n && i < 8; i++) out[i] = h[i];
  unsigned long long z[8] = {0};
  return hipMemcpyToSymbol(HIP_SYMBOL(g_cnt), z, sizeof(z)) == hipSuccess ? 0 : -1;
}
#endif
#ifdef MHQ_DIAG_TIMELINE
extern "C" int mhq_diag_timeline(unsigned long long *out, int n) {
  const int m = n < 1024 * 16 * kTlSlots ? n : 1024 * 16 * kTlSlots;
  return hipMemcpyFromSymbol(out, HIP_SYMBOL(g_tl), m * sizeof(unsigned long long)) == hipSuccess ? kTlSlots : -1;
}
#endif

hipError_t launch_decode(const DevTables &t, const uint8_t *in, const uint64_t *in_off, uint64_t in_bias,
                         uint64_t n, uint8_t *out, const uint64_t *out_off, uint64_t out_bias,
                         uint32_t *out_len, uint8_t *status, hipStream_t s, const uint32_t *in_end,
                         const StrFinish *str) {
  if (n == 0) return hipSuccess;
  // One workgroup per CU, each a contiguous range of whole wave tiles.  The
  // tile length (<= kTile) is chosen so that every wave gets the same number
  // of tiles: no wave idles through a last, partial round.  (A shorter first
  // round of tiles, 86 + 128 + 128 literals per wave on the north star instead
  // of 3 x 114, was 1 us slower: the opening does not shorten with its bytes.)
  const uint64_t cus = (uint64_t)dev::device_cus();
  const uint64_t slots = cus * kWaves;
  const uint64_t rounds = (n + slots * kTile - 1) / (slots * kTile) + MHQ_DEC_XROUNDS;
  const uint64_t tl = std::max<uint64_t>(1, (n + slots * rounds - 1) / (slots * rounds));
  const uint64_t per_block = (((n + cus - 1) / cus + tl - 1) / tl) * tl;
  const unsigned grid = (unsigned)((n + per_block - 1) / per_block);
  if (in_end)
    decode_kernel<true><<<dim3(grid), dim3(kT), 0, s>>>(in, in_off, in_end, str ? *str : StrFinish{}, in_bias, n, out,
                                                        out_off, out_bias,
                                                        out_len, status, t.lut1, t.lut2, t.len, per_block,
                                                        (uint32_t)tl);
  else
    decode_kernel<false><<<dim3(grid), dim3(kT), 0, s>>>(in, in_off, nullptr, StrFinish{}, in_bias, n, out, out_off,
                                                         out_bias,
                                                         out_len, status, t.lut1, t.lut2, t.len, per_block,
                                                         (uint32_t)tl);
  return hipGetLastError();
}

// The decode's grid and tile length (launch_decode), the tile length cut to
// what fits the slices at the block's mean frame (decode_kernel's kGaps rule).
hipError_t launch_read_fused(const DevTables &t, const uint8_t *blk, uint64_t blk_len, const uint64_t *pos,
                             const uint64_t *limit, const uint8_t *prefix, uint64_t n, uint8_t *out,
                             uint64_t *out_off, uint32_t *out_len, uint8_t *status, uint64_t *next,
                             uint64_t *sc_start, uint32_t *sc_hend, uint8_t *sc_kind, uint64_t *fallback,
                             uint64_t gen, hipStream_t s) {
  if (n == 0) return hipSuccess;
  const uint64_t cus = (uint64_t)dev::device_cus();
  const uint64_t slots = cus * kWaves;
  const uint64_t rounds = (n + slots * kTile - 1) / (slots * kTile) + MHQ_DEC_XROUNDS;
  uint64_t tl = std::max<uint64_t>(1, (n + slots * rounds - 1) / (slots * rounds));
  const uint64_t nout = blk_len / 5 * 8 + (blk_len % 5) * 8 / 5;
  const uint64_t ain = (blk_len + n - 1) / n, aout = (nout + n - 1) / n;
  const uint64_t fit = std::min((uint64_t)(kWIn - 16) * 5u / (6u * ain + 10u),
                                (uint64_t)(kWOut - 16) * 5u / (6u * aout + 10u));
  if (fit >= (uint64_t)kWave && fit < tl) tl = fit;
  const uint64_t per_block = (((n + cus - 1) / cus + tl - 1) / tl) * tl;
  const unsigned grid = (unsigned)((n + per_block - 1) / per_block);
  RsArgs a{blk, blk_len, pos, limit, prefix, n, out, out_off, next, out_len, status, sc_start, sc_hend, sc_kind,
           fallback, gen};
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
  const uint64_t rounds = (n + slots * kTile - 1) / (slots * kTile) + MHQ_DEC_XROUNDS;
  const uint64_t tl = std::max<uint64_t>(1, (n + slots * rounds - 1) / (slots * rounds));
  const uint64_t per_block = (((n + cus - 1) / cus + tl - 1) / tl) * tl;
  const unsigned grid = (unsigned)((n + per_block - 1) / per_block);
  if (grid > kReadFallbackMaxWgs) return hipErrorInvalidConfiguration;
  RsFallback f{RsArgs{blk, blk_len, pos, limit, prefix, n, out, out_off, next, out_len, status, sc_start, sc_hend,
                      sc_kind, fallback, gen},
               out_cap, wg_agg, wg_fin};
  read_fallback_kernel<<<dim3(grid), dim3(kT), 0, s>>>(f, t.lut1, t.lut2, t.len, per_block, (uint32_t)tl);
  return hipGetLastError();
}

}  // namespace mhq
