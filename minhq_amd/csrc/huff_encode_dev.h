// huff_encode_dev.h -- device core of the gfx950 batch encode (tables in LDS,
// the staged bit writer, the per-literal encode), shared by the encode kernels
// (huff_encode.hip) and the one-launch packed encode (enc_packed.hip).  The
// design is described in huff_encode.hip.
#pragma once
#include <hip/hip_runtime.h>
#include <stdlib.h>
#include <string.h>

#include <algorithm>

#include "huff_common.h"
#include "huff_kernels.h"
#include "huff_table.h"

#ifndef MHQ_ENC_T  // threads (= literals) per block tile
#define MHQ_ENC_T 512
#endif
#ifndef MHQ_ENC_INCAP  // plaintext staging slice (bytes)
#define MHQ_ENC_INCAP 24576
#endif
#ifndef MHQ_ENC_OUTCAP  // output staging slice (bytes, encode only)
#define MHQ_ENC_OUTCAP 20480
#endif
#ifndef MHQ_ENC_NTST  // encode_len's lengths and the cooperative encode's whole chunks as streaming stores (config 5 encode 162.8 -> 154.9 us)
#define MHQ_ENC_NTST 1
#endif
#ifndef MHQ_LEN_LPL  // encode_len: literals per lane (2: 76 VGPRs, 6 waves per SIMD, 5 % slower)
#define MHQ_LEN_LPL 1
#endif
#ifndef MHQ_ENC_BLOCKS  // resident workgroups per CU
#define MHQ_ENC_BLOCKS 3
#endif
#ifndef MHQ_ENC_SHORT_MEAN  // mean plaintext bytes up to which the thread form encodes (96 since r05ai: 40-96 B -16..-38 %)
#define MHQ_ENC_SHORT_MEAN 96
#endif
#ifndef MHQ_ENC_SHORT_GENS  // resident generations of the short form's grid before its workgroups loop over ranges
#define MHQ_ENC_SHORT_GENS 4
#endif
#ifndef MHQ_ENC_TINY_MEAN  // mean plaintext bytes up to which the cooperative kernel encodes (per-literal costs)
#define MHQ_ENC_TINY_MEAN 20
#endif

namespace mhq {
namespace {

using namespace dev;

constexpr int kT = MHQ_ENC_T;
constexpr int kInCap = MHQ_ENC_INCAP;
constexpr int kOutCap = MHQ_ENC_OUTCAP;
constexpr int kPF = (kInCap / 16 + kT - 1) / kT;  // prefetched input chunks per thread
constexpr int kBuckets = 64;
constexpr uint32_t kShortMean = MHQ_ENC_SHORT_MEAN;
constexpr uint32_t kTinyMean = MHQ_ENC_TINY_MEAN;
// The thread-per-literal kernel's batches: a mean literal over kTinyMean and
// up to kShortMean bytes (config 2, the north star, config 4's Zipf text --
// 169 against 189 us at 2^22 -- and text up to a 96-B mean: -16 to -38 %,
// profiles/r05ai_encode_forms.txt); the cooperative kernel takes the rest
// (shorter: config 3's QIF literals, 26.6 us against 38.3; longer: config
// 5's long codes, 158 against 331 us).
__device__ __forceinline__ bool thread_form(uint64_t bytes, uint64_t n) {
  return bytes > (uint64_t)kTinyMean * n && bytes <= (uint64_t)kShortMean * n;
}

#ifndef MHQ_ENC_PERSIST_MEAN  // the thread kernel's persistent ranges above this mean literal (bytes; one range of kT literals per workgroup below)
#define MHQ_ENC_PERSIST_MEAN 40
#endif
#ifndef MHQ_ENC_QUAD  // the thread kernel puts a staged word's four codes at once when they fit 32 bits
#define MHQ_ENC_QUAD 1
#endif
#ifndef MHQ_ENC_GW  // 1: literals encoded straight from global memory read aligned dwords (encode_literal_global)
#define MHQ_ENC_GW 1
#endif
#ifndef MHQ_ENC_ALIGN  // the thread kernel's LDS alignment (16: its 16-B LDS accesses are single ds_*_b128)
#define MHQ_ENC_ALIGN 16
#endif
template <bool kEmit>
struct alignas(MHQ_ENC_ALIGN) Smem {
  uint2 code[256];                // (code right-justified, length)
  uint32_t in_w[kInCap / 4 + 4];  // plaintext, natural byte order
  uint32_t out_w[kEmit ? kOutCap / 4 + 4 : 4];  // output staging (global layout, zero-filled)
  uint32_t rec[kT + 1];           // per boundary: input byte index | output byte index << 16
  uint16_t order[kT];             // literals by ascending plaintext length
  uint32_t hist[kBuckets];
  uint64_t nbase[2];              // in_off / out_off at the next sub-tile's first literal
};

// Bit writer into the zeroed LDS staging words ow[]: complete words are OR-ed
// in big-endian byte order; bits before the literal's first byte are zero, so
// a word shared with the previous literal takes only this literal's bits.
struct BitOut {
  uint32_t *ow;
  uint32_t wpos;   // index of the word being filled
  uint32_t nbits;  // bits pending in acc (its low nbits bits), counting the zero prefix
  uint64_t acc;

  __device__ __forceinline__ void init(uint32_t *ow_, uint32_t start) {
    ow = ow_;
    wpos = start >> 2;
    nbits = (start & 3u) * 8u;
    acc = 0;
  }
  __device__ __forceinline__ void put(uint32_t code, uint32_t len) {
    acc = (acc << len) | code;
    nbits += len;
    // branch free: some lane of the wave completes a word at nearly every
    // byte, so the OR is issued anyway; the others OR 0 into their own word
    // (a per-code branch: config 2 +1 %, north star +0.7 to 1.3 %, r04e)
    const bool full = nbits >= 32u;
    nbits -= full ? 32u : 0u;
    atomicOr(&ow[wpos], full ? __builtin_bswap32((uint32_t)(acc >> nbits)) : 0u);
    wpos += full ? 1u : 0u;
  }
  // Pad with 1 bits to an octet boundary (bitWriter.Pad(0xff)) and OR out the rest.
  __device__ __forceinline__ void finish() {
    const uint32_t padn = (8u - (nbits & 7u)) & 7u;
    acc = (acc << padn) | ((1u << padn) - 1u);
    nbits += padn;
    if (nbits) atomicOr(&ow[wpos], __builtin_bswap32((uint32_t)(acc << (32u - nbits))));
  }
};

// Bit writer over global bytes (literals encoded straight from global memory):
// byte by byte.
struct BitOutGlobal {
  uint8_t *o;
  uint32_t nbits;
  uint64_t acc;
  __device__ __forceinline__ void put(uint32_t code, uint32_t len) {
    acc = (acc << len) | code;
    nbits += len;
    while (nbits >= 8u) {
      nbits -= 8u;
      *o++ = (uint8_t)(acc >> nbits);
    }
  }
  __device__ __forceinline__ void finish() {
    if (nbits) *o = (uint8_t)((acc << (8u - nbits)) | (0xffu >> nbits));
  }
};

// One literal, one thread, straight from global memory (literals larger than
// the staging slice).
template <bool kEmit>
__device__ void encode_literal_global(const uint8_t *src, uint64_t nbytes, uint8_t *dst, const uint2 *code,
                                      uint32_t *enc_len) {
  uint64_t bits = 0;
  BitOutGlobal bo{dst, 0, 0};
  const uint8_t *p = src, *e = src + nbytes;
#if MHQ_ENC_GW
  // whole aligned dwords between a byte-wise head and tail
  for (; p < e && ((uintptr_t)p & 3u); p++) {
    const uint2 c = code[*p];
    bits += c.y;
    if (kEmit) bo.put(c.x, c.y);
  }
  for (; p + 4 <= e; p += 4) {
    const uint32_t w = *(const uint32_t *)p;
#pragma unroll
    for (int k = 0; k < 4; k++) {
      const uint2 c = code[(w >> (8 * k)) & 0xffu];
      bits += c.y;
      if (kEmit) bo.put(c.x, c.y);
    }
  }
#endif
  for (; p < e; p++) {
    const uint2 c = code[*p];
    bits += c.y;
    if (kEmit) bo.put(c.x, c.y);
  }
  if (kEmit) bo.finish();
  if (!kEmit) *enc_len = (uint32_t)((bits + 7u) / 8u);
}

// Encodes staged plaintext bytes [p, e); returns the encoded bit count.
// Per staged word: its four code lookups are issued together and the next
// word is read ahead, so a word costs one LDS round trip, not one per byte.
// Only the literal's first and last words hold bytes outside [p, e) (they
// look up harmlessly and are masked to nothing); the words between them are
// put without the per-byte range tests (MHQ_ENC_MIDLOOP).
#ifndef MHQ_ENC_MIDLOOP
#define MHQ_ENC_MIDLOOP 1
#endif
template <bool kEmit, bool kMasked, class SM>
__device__ __forceinline__ void encode_word(const SM &sm, uint32_t w, uint32_t q, uint32_t p, uint32_t e,
                                            BitOut &bo, uint32_t &bits) {
  uint2 c[4];
#pragma unroll
  for (int b = 0; b < 4; b++) c[b] = sm.code[(w >> (8 * b)) & 0xffu];
  uint32_t len[4], code[4];
#pragma unroll
  for (int b = 0; b < 4; b++) {
    const uint32_t x = q + (uint32_t)b;
    const bool in = !kMasked || (x >= p && x < e);
    len[b] = in ? c[b].y : 0u;
    code[b] = in ? c[b].x : 0u;
  }
  const uint32_t l4 = len[0] + len[1] + len[2] + len[3];
  bits += l4;
#if MHQ_ENC_QUAD
  // The word's four codes as one put when they fit 32 bits (text: nearly
  // always): one LDS OR per word instead of one per byte.
  if (kEmit) {
    if (l4 <= 32u) {
      uint32_t cc = code[0];
#pragma unroll
      for (int b = 1; b < 4; b++) cc = (cc << len[b]) | code[b];
      bo.put(cc, l4);
    } else {
#pragma unroll
      for (int b = 0; b < 4; b++) bo.put(code[b], len[b]);
    }
  }
#else
  if (kEmit) {
#pragma unroll
    for (int b = 0; b < 4; b++) bo.put(code[b], len[b]);
  }
#endif
}

template <bool kEmit, class SM>
__device__ __forceinline__ uint32_t encode_one(SM &sm, uint32_t p, uint32_t e, uint32_t ostart) {
  uint32_t bits = 0;
  BitOut bo;
  if (kEmit) bo.init(sm.out_w, ostart);
  uint32_t q = p & ~3u;
  uint32_t w = sm.in_w[q >> 2];
#if MHQ_ENC_MIDLOOP
  if (q < e) {
    // the first word (bytes before p), then whole words, then the last partial word
    uint32_t wn = sm.in_w[(q >> 2) + 1u];  // in_w has slack words past the slice
    encode_word<kEmit, true>(sm, w, q, p, e, bo, bits);
    w = wn;
    q += 4u;
    for (; q + 4u <= e; q += 4u) {
      wn = sm.in_w[(q >> 2) + 1u];
      encode_word<kEmit, false>(sm, w, q, p, e, bo, bits);
      w = wn;
    }
    if (q < e) encode_word<kEmit, true>(sm, w, q, p, e, bo, bits);
  }
#else
  for (; q < e; q += 4u) {
    const uint32_t wn = sm.in_w[(q >> 2) + 1u];  // in_w has slack words past the slice
    encode_word<kEmit, true>(sm, w, q, p, e, bo, bits);
    w = wn;
  }
#endif
  if (kEmit) bo.finish();
  return bits;
}

// ---- a block's literals: one contiguous range, greedy sub-tiles ----------
// As in huff_decode.hip: block b owns literals [b*R, (b+1)*R); a sub-tile is
// the longest run of at most kT literals that fits the slices; the next
// sub-tile's offsets and plaintext are loaded into registers while this one
// is encoded (raw values only, unconditional loads), and a sub-tile's output
// is stored only after the next sub-tile's loads have been issued.

__device__ __forceinline__ uint32_t vzero() {
  uint32_t z;
  asm volatile("v_mov_b32 %0, 0" : "=v"(z));
  return z;
}

__device__ __forceinline__ uint64_t vload(const uint64_t *__restrict__ p, uint64_t i) { return p[i + vzero()]; }

// The builtin returns int: each half goes through uint32_t, or a low word
// >= 2^31 would sign-extend over the high one (offsets of 2-4 GiB, 6-8 GiB...).
__device__ __forceinline__ uint64_t uniform64(uint64_t v) {
  return (uint64_t)(uint32_t)__builtin_amdgcn_readfirstlane((uint32_t)v) |
         ((uint64_t)(uint32_t)__builtin_amdgcn_readfirstlane((uint32_t)(v >> 32)) << 32);
}

struct Next {           // raw loads for the sub-tile that starts at literal `cur`
  uint64_t ie64, oe64;  // in_off / out_off at the end of literal cur + min(tid, cnt-1)
  u32x4 v[kPF];         // plaintext chunk min(tid + kT*k, chunks-1) from the 16-B aligned start
};

__device__ __forceinline__ uint32_t prefetch_chunks(const uint8_t *in, uint64_t in_bias, uint64_t ic, uint64_t iend) {
  const uint32_t delta = (uint32_t)((uintptr_t)(in + (ic - in_bias)) & 15u);
  return (uint32_t)min(((iend - ic) + delta + 15u) >> 4, (uint64_t)(kInCap / 16));
}

template <bool kEmit>
__device__ __forceinline__ void issue_next(Next &nx, const uint8_t *__restrict__ in, uint64_t in_bias,
                                           const uint64_t *__restrict__ in_off,
                                           const uint64_t *__restrict__ out_off, uint64_t cur, uint64_t lim,
                                           uint64_t ic, uint64_t iend, uint32_t tid) {
  const uint64_t j = min(cur + 1u + tid, lim);
  nx.ie64 = in_off[j];
  if (kEmit) nx.oe64 = out_off[j];
  const uint8_t *a = in + (ic - in_bias);
  const u32x4 *src = (const u32x4 *)(a - ((uintptr_t)a & 15u));
  const uint32_t chunks = prefetch_chunks(in, in_bias, ic, iend);
  if (chunks == 0) return;  // nothing left: the aligned chunk at the end may lie past the buffer
#pragma unroll
  for (int k = 0; k < kPF; k++) {
    const uint32_t c = min(tid + (uint32_t)kT * k, chunks - 1u);
    nx.v[k] = __builtin_nontemporal_load(src + c);  // aligned, holds a valid byte: never crosses a page
  }
}

}  // namespace
}  // namespace mhq
