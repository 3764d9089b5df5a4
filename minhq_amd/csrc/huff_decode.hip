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
// Structure: one workgroup of kT threads owns a block tile of kT consecutive
// literals and decodes it with one thread per literal.
//   * staging: the tile's offsets (one coalesced u64 per thread), its input
//     bytes (aligned 16-B loads, byte-swapped, reverse word order so that the
//     logical word pair {k+1, k} is one little-endian u64) and its output
//     region (zero-filled, global layout) live in LDS; the output leaves as
//     aligned 16-B stores, out_len/status as coalesced stores;
//   * balance: a counting sort by encoded length gives thread t the literal
//     of rank t, so the 64 literals of a wave have similar lengths and the
//     wave's loop runs about as long as its average literal;
//   * occupancy: two workgroups per CU (2 x kT/64 waves) hide the LDS round
//     trips of the per-literal decode chains;
//   * a probe reads LUT1 with the next 12 bits (one or two codes of <= 12
//     bits) or, for longer codes, LUT2 by count of leading ones; output bytes
//     are packed into registers on the LDS word grid and OR-ed into the zeroed
//     staging words, so literals that share a word need no ordering.
//   * a tile whose bytes exceed the staging slices is processed as several
//     sub-tiles; a single literal larger than a slice is decoded by one
//     thread straight from global memory.
#include <hip/hip_runtime.h>

#include "huff_common.h"
#include "huff_kernels.h"
#include "huff_table.h"

#ifndef MHQ_DEC_T  // threads per block, literals per thread, and the staging slices
#define MHQ_DEC_T 384
#define MHQ_DEC_LPT 2
#define MHQ_DEC_INCAP 20480
#define MHQ_DEC_OUTCAP 30720
#endif
#ifndef MHQ_DEC_BLOCKS  // resident workgroups per CU
#define MHQ_DEC_BLOCKS 2
#endif

namespace mhq {
namespace {

using namespace dev;

constexpr int kT = MHQ_DEC_T;
constexpr int kLPT = MHQ_DEC_LPT;  // 1 or 2
constexpr int kL = kT * kLPT;      // literals per block tile
constexpr int kInCap = MHQ_DEC_INCAP;    // staged input bytes (incl. 16-B alignment slack)
constexpr int kOutCap = MHQ_DEC_OUTCAP;  // staged output bytes
constexpr uint32_t kInWords = kInCap / 4 + 4;
constexpr int kBuckets = 64;

struct Smem {
  uint32_t lut1[kLut1Size];
  uint16_t lut2[kLut2Size];
  uint32_t in_w[kInWords];          // stream words, byte-swapped, reverse word order
  uint32_t out_w[kOutCap / 4 + 4];  // output staging (global layout, zero-filled)
  uint2 rec[kL + 1];                // per boundary: (input byte index, output byte index)
  uint32_t olen[kL];                // out_len | status << 31
  uint16_t order[kL];               // literals by ascending encoded length
  uint32_t hist[kBuckets];
  uint64_t base[2];                 // the sub-tile's in_off / out_off at its first literal
};

// One literal, one thread, straight from global memory: literals too large for
// the staging slices.  Same decision rules as the staged loop.
__device__ void decode_literal_global(const uint8_t *src, uint64_t nbytes, uint8_t *dst, uint64_t cap,
                                      const uint32_t *lut1, const uint16_t *lut2, uint32_t *out_len,
                                      uint8_t *status) {
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
    const uint32_t e = lut1[win >> (32 - kLut1Bits)];
    const uint32_t nsym = e >> 26;
    if (nsym == 0) {
      const uint32_t nw = ~win;
      const uint32_t c = nw ? (uint32_t)__builtin_clz(nw) : 32u;
      if (c >= (uint32_t)kEosOnes) {
        st = rem > (uint64_t)kEosOnes;
        break;
      }
      const uint32_t e2 = lut2[(c << kLut2SubBits) | ((win << (c + 1)) >> (32 - kLut2SubBits))];
      const uint32_t L = e2 >> 8;
      if (L == 0 || L > rem) break;
      dst[n++] = (uint8_t)e2;
      p += L;
      continue;
    }
    const uint32_t len0 = (e >> 16) & 31u, tot = (e >> 21) & 31u;
    if (len0 > rem) break;
    dst[n++] = (uint8_t)e;
    if (nsym == 2 && tot <= rem && n < cap) {
      dst[n++] = (uint8_t)(e >> 8);
      p += tot;
    } else {
      p += len0;
    }
  }
  *out_len = (uint32_t)n;
  *status = st;
}

#ifdef MHQ_DEC_WINDOW
// The 32 stream bits at bit position p (one ds_read2_b32 of logical words k, k+1).
__device__ __forceinline__ uint32_t window_at(const uint32_t *in_w, uint32_t p) {
  const uint32_t k = p >> 5, sh = p & 31u;
  const uint32_t *wp = in_w + (kInWords - 2u - k);
  const uint64_t ww = (uint64_t)wp[0] | ((uint64_t)wp[1] << 32);  // {word k+1, word k}
  return (uint32_t)((ww << sh) >> 32);
}
#endif

// Decodes staged literal bits [p, endbit) into staging bytes [optr, oend).
// Returns out_len | status << 31.
__device__ __forceinline__ uint32_t decode_one(Smem &sm, uint32_t p, uint32_t endbit, uint32_t optr,
                                               uint32_t oend) {
  const uint32_t ostart = optr;
  uint32_t acc = 0;  // this literal's bytes of word optr>>2 below optr
  uint32_t bad = 0;
  bool fin = false;
#ifndef MHQ_DEC_WINDOW
  // 64-bit bit buffer: the next nb >= 32 stream bits, MSB first.  The refill
  // word is read ahead of each probe, so a probe waits on one LDS round trip
  // (its LUT entry) instead of two.
  uint32_t rem = endbit - p;
  uint32_t nxt = (p >> 5) + 2u;  // logical index of the next word to load
  uint64_t bb = ((uint64_t)sm.in_w[kInWords - 1u - (p >> 5)] << 32 | sm.in_w[kInWords - 2u - (p >> 5)])
                << (p & 31u);
  uint32_t nb = 64u - (p & 31u);
#endif
  while (!fin) {
    const uint32_t w0 = optr >> 2;
    uint64_t o64 = acc;
#pragma unroll
    for (int u = 0; u < 2; u++) {  // two probes per output flush
#ifdef MHQ_DEC_WINDOW
      const uint32_t win = window_at(sm.in_w, p);
      const uint32_t rem = endbit - p;
#else
      const uint32_t win = (uint32_t)(bb >> 32);
      const uint32_t wnext = sm.in_w[kInWords - 1u - nxt];
#endif
      const uint32_t e = sm.lut1[win >> (32 - kLut1Bits)];
      uint32_t len0 = (e >> 16) & 31u, tot = (e >> 21) & 31u, ns = e >> 26, syms = e & 0xffffu;
      if (ns == 0) {  // a code of 13..30 bits, or the all-ones EOS prefix
        const uint32_t nw = ~win;
        const uint32_t c = nw ? (uint32_t)__builtin_clz(nw) : 32u;
        if (c >= (uint32_t)kEosOnes) {
          len0 = tot = 0xffffffffu;         // never fits: the literal ends here
          bad |= rem > (uint32_t)kEosOnes;  // a 31st bit exists: nil child
        } else {
          const uint32_t e2 = sm.lut2[(c << kLut2SubBits) | ((win << (c + 1)) >> (32 - kLut2SubBits))];
          len0 = tot = (e2 >> 8) ? (e2 >> 8) : 0xffffffffu;
          ns = 1;
          syms = e2 & 0xffu;
        }
      }
      const bool ct = tot <= rem;
      uint32_t cnt = ct ? ns : (len0 <= rem ? 1u : 0u);
      const uint32_t room = oend - optr;  // Read() stops once p is full (hc/huffman.go:104)
      cnt = cnt < room ? cnt : room;
      cnt = fin ? 0u : cnt;
      o64 |= (uint64_t)__builtin_amdgcn_ubfe(syms, 0, cnt * 8u) << ((optr - 4u * w0) * 8u);
      optr += cnt;
      const uint32_t used = cnt ? (ct ? tot : len0) : 0u;
#ifdef MHQ_DEC_WINDOW
      p += used;
#else
      rem -= used;
      bb <<= used;
      nb -= used;
      if (nb < 32u) {  // nb >= 2 here: a probe consumes at most 30 bits
        bb |= (uint64_t)wnext << (32u - nb);
        nb += 32u;
        nxt++;
      }
#endif
      fin |= cnt == 0;
    }
    if (o64) {
      atomicOr(&sm.out_w[w0], (uint32_t)o64);
      atomicOr(&sm.out_w[w0 + 1], (uint32_t)(o64 >> 32));
    }
    acc = (optr >> 2) != w0 ? (uint32_t)(o64 >> 32) : (uint32_t)o64;
  }
  bad = optr != oend ? bad : 0u;
  return (optr - ostart) | (bad << 31);
}

__global__ __launch_bounds__(kT) void decode_kernel(
    const uint8_t *__restrict__ in, const uint64_t *__restrict__ in_off, uint64_t in_bias, uint64_t n,
    uint8_t *__restrict__ out, const uint64_t *__restrict__ out_off, uint64_t out_bias,
    uint32_t *__restrict__ out_len, uint8_t *__restrict__ status, const uint32_t *__restrict__ g_lut1,
    const uint16_t *__restrict__ g_lut2, uint64_t ntiles) {
  __shared__ Smem sm;
  const uint32_t tid = threadIdx.x;
  const uint32_t lane = tid % kWave;
  const uint32_t wave = tid / kWave;
  for (uint32_t i = tid; i < kLut1Size / 4; i += kT) ((u32x4 *)sm.lut1)[i] = ((const u32x4 *)g_lut1)[i];
  for (uint32_t i = tid; i < kLut2Size / 8; i += kT) ((u32x4 *)sm.lut2)[i] = ((const u32x4 *)g_lut2)[i];

  for (uint64_t t = blockIdx.x; t < ntiles; t += gridDim.x) {
    const uint64_t s = t * kL;
    const uint32_t cnt = (uint32_t)min((uint64_t)kL, n - s);
    // end boundaries of literals tid + kT*j (coalesced u64 loads)
    uint64_t ie[kLPT], oe[kLPT];
#pragma unroll
    for (int j = 0; j < kLPT; j++) {
      const uint32_t l = tid + kT * j;
      ie[j] = l < cnt ? in_off[s + l + 1] : 0;
      oe[j] = l < cnt ? out_off[s + l + 1] : 0;
    }
    uint32_t cur = 0;
    while (cur < cnt) {
      __syncthreads();  // the previous sub-tile is fully consumed
      if (cur == 0 && tid == 0) {
        sm.base[0] = in_off[s];
        sm.base[1] = out_off[s];
      }
#pragma unroll
      for (int j = 0; j < kLPT; j++) {
        if (cur != 0 && tid + kT * j == cur - 1) {
          sm.base[0] = ie[j];
          sm.base[1] = oe[j];
        }
      }
      __syncthreads();
      const uint64_t ic = sm.base[0], oc = sm.base[1];
      const uint8_t *ia = in + (ic - in_bias);
      uint8_t *oa = out + (oc - out_bias);
      const uint32_t idelta = (uint32_t)((uintptr_t)ia & 15u);
      const uint32_t odelta = (uint32_t)((uintptr_t)oa & 15u);
      // a literal joins the sub-tile when both slices hold everything up to its end
      bool fits[kLPT];
      uint32_t nfit = 0;
#pragma unroll
      for (int j = 0; j < kLPT; j++) {
        const uint32_t l = tid + kT * j;
        fits[j] = l < cnt && l >= cur && (ie[j] - ic) + idelta <= (uint64_t)kInCap &&
                  (oe[j] - oc) + odelta <= (uint64_t)kOutCap;
        nfit += (uint32_t)__syncthreads_count(fits[j]);
      }
      const uint32_t end = cur + nfit;
      if (end == cur) {  // one literal larger than the slices
        if (tid == 0)
          decode_literal_global(ia, in_off[s + cur + 1] - ic, oa, out_off[s + cur + 1] - oc, sm.lut1, sm.lut2,
                                out_len + s + cur, status + s + cur);
        cur++;
        continue;
      }
      const uint32_t m = end - cur;
      if (tid == 0) sm.rec[0] = make_uint2(idelta, odelta);
#pragma unroll
      for (int j = 0; j < kLPT; j++)
        if (fits[j])
          sm.rec[tid + kT * j - cur + 1] =
              make_uint2((uint32_t)(ie[j] - ic) + idelta, (uint32_t)(oe[j] - oc) + odelta);
      if (tid < kBuckets) sm.hist[tid] = 0;
      __syncthreads();
      const uint32_t in_bytes = sm.rec[m].x, out_bytes = sm.rec[m].y;
      // stage the input (byte-swapped, reverse word order); zero the output slice
      {
        const uint32_t chunks = (in_bytes + 15u) >> 4;
        const u32x4 *src = (const u32x4 *)(ia - idelta);
        for (uint32_t c = tid; c < chunks; c += kT) {
          u32x4 v = __builtin_nontemporal_load(src + c);  // aligned: never crosses a page
          v.x = __builtin_bswap32(v.x);
          v.y = __builtin_bswap32(v.y);
          v.z = __builtin_bswap32(v.z);
          v.w = __builtin_bswap32(v.w);
          *(u32x4 *)(sm.in_w + kInWords - 4u - 4u * c) = v.wzyx;
        }
        const uint32_t ochunks = (out_bytes + 15u) >> 4;
        for (uint32_t c = tid; c < ochunks; c += kT) *(u32x4 *)(sm.out_w + 4u * c) = u32x4{0u, 0u, 0u, 0u};
      }
      // counting sort by encoded length
      uint32_t bk[kLPT], rk[kLPT];
#pragma unroll
      for (int j = 0; j < kLPT; j++) {
        const uint32_t l = tid + kT * j;
        bk[j] = 0;
        rk[j] = 0;
        if (l < m) {
          const uint32_t bytes = sm.rec[l + 1].x - sm.rec[l].x;
          bk[j] = bytes < 32u ? bytes : min(32u + ((bytes - 32u) >> 4), (uint32_t)kBuckets - 1u);
          rk[j] = atomicAdd(&sm.hist[bk[j]], 1u);
        }
      }
      __syncthreads();
      if (wave == 0) {  // exclusive scan of the bucket counts
        const uint32_t h = sm.hist[lane];
        uint32_t x = h;
#pragma unroll
        for (int d = 1; d < kWave; d <<= 1) {
          const uint32_t y = __shfl_up(x, d);
          if ((int)lane >= d) x += y;
        }
        sm.hist[lane] = x - h;
      }
      __syncthreads();
#pragma unroll
      for (int j = 0; j < kLPT; j++)
        if (tid + kT * j < m) sm.order[sm.hist[bk[j]] + rk[j]] = (uint16_t)(tid + kT * j);
      __syncthreads();
      // thread t decodes the literals of rank t and (with two per thread) m-1-t:
      // short + long pairs, so every lane's work is about the same
#pragma unroll
      for (int j = 0; j < kLPT; j++) {
        const uint32_t r = j == 0 ? tid : m - 1u - tid;
        const bool mine = kLPT == 1 ? tid < m : (j == 0 ? tid < (m + 1u) / 2u : tid < m / 2u);
        if (mine) {
          const uint32_t lit = sm.order[r];
          const uint2 r0 = sm.rec[lit], r1 = sm.rec[lit + 1];
#ifdef MHQ_DIAG_NO_DECODE  // diagnostic build: staging and stores only
          sm.olen[lit] = 0;
#else
          sm.olen[lit] = decode_one(sm, r0.x * 8u, r1.x * 8u, r0.y, r1.y);
#endif
        }
      }
      __syncthreads();
      store_out(oa - odelta, (const uint8_t *)sm.out_w, odelta, out_bytes, tid, kT);
#pragma unroll
      for (int j = 0; j < kLPT; j++) {
        const uint32_t l = tid + kT * j;
        if (l < m) {
          const uint32_t v = sm.olen[l];
          out_len[s + cur + l] = v & 0x7fffffffu;
          status[s + cur + l] = (uint8_t)(v >> 31);
        }
      }
      cur = end;
    }
  }
}

}  // namespace

hipError_t launch_decode(const DevTables &t, const uint8_t *in, const uint64_t *in_off, uint64_t in_bias,
                         uint64_t n, uint8_t *out, const uint64_t *out_off, uint64_t out_bias,
                         uint32_t *out_len, uint8_t *status, hipStream_t s) {
  if (n == 0) return hipSuccess;
  const uint64_t ntiles = (n + kL - 1) / kL;
  decode_kernel<<<dim3(dev::tile_grid(ntiles, 1, MHQ_DEC_BLOCKS * MHQ_PER_CU)), dim3(kT), 0, s>>>(
      in, in_off, in_bias, n, out, out_off, out_bias, out_len, status, t.lut1, t.lut2, ntiles);
  return hipGetLastError();
}

}  // namespace mhq
