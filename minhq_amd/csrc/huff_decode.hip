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
// Structure (one workgroup = kWaves wave64s, LUT1/LUT2 shared in LDS):
//   * each wave walks tiles of kTileLits literals; a tile is staged in the
//     wave's LDS slice (offsets -> boundary records; input bytes byte-swapped
//     and in reverse word order, so a pair of logical words {k+1, k} is one
//     little-endian u64), decoded, and its output region written back with
//     aligned 16-B stores;
//   * load balance: a counting sort by encoded length orders the tile's
//     literals; stream k (two per lane) takes ranks k, 2K-1-k, 2K+k, ...
//     ("snake"), so every stream gets about the same number of bits;
//   * a stream keeps its bits in a 64-bit register buffer refilled one word at
//     a time from a prefetched LDS word, so the only LDS round trip on the
//     decode chain is the LUT probe; the two streams of a lane are advanced
//     in the same straight-line blocks so their probes overlap;
//   * a probe reads LUT1 with the next 12 bits (one or two codes of <= 12
//     bits) or, for longer codes, LUT2 by count of leading ones; output bytes
//     are packed into registers on the LDS word grid and OR-ed into the zeroed
//     staging words, so literals that share a word need no ordering.
#include <hip/hip_runtime.h>

#include "huff_common.h"
#include "huff_kernels.h"
#include "huff_table.h"

#ifndef MHQ_DEC_WAVES  // geometry (measured on MI355X: 16 waves/CU x 128-literal tiles is fastest)
#define MHQ_DEC_WAVES 16
#define MHQ_DEC_TILE 128
#define MHQ_DEC_INCAP 3072
#define MHQ_DEC_OUTCAP 3840
#endif

namespace mhq {
namespace {

using namespace dev;

constexpr int kWaves = MHQ_DEC_WAVES;
constexpr int kThreads = kWave * kWaves;
constexpr int kTileLits = MHQ_DEC_TILE;
constexpr int kInCap = MHQ_DEC_INCAP;    // staged input bytes per wave (incl. 16-B alignment slack)
constexpr int kOutCap = MHQ_DEC_OUTCAP;  // staged output bytes per wave
constexpr uint32_t kInWords = kInCap / 4 + 4;
#ifndef MHQ_DEC_STREAMS
#define MHQ_DEC_STREAMS 1
#endif
constexpr int kStreams = MHQ_DEC_STREAMS;  // per lane (1 or 2)
constexpr uint32_t kK = kWave * kStreams;
constexpr int kBuckets = 64;
constexpr uint32_t kNone = 0xffffffffu;
constexpr int kPer = (kTileLits + kWave - 1) / kWave;

struct WaveSmem {
  uint32_t in_w[kInWords];         // stream words, byte-swapped, reverse word order
  uint32_t out_w[kOutCap / 4 + 4]; // output staging (global layout, zero-filled)
  uint2 rec[kTileLits + 2];        // per boundary: (input byte index, output byte index)
  uint32_t olen[kTileLits];        // out_len | status << 31
  uint16_t order[kTileLits];       // literals by ascending encoded length
  uint32_t hist[kBuckets];
};
struct Smem {
  uint32_t lut1[kLut1Size];
  uint16_t lut2[kLut2Size];
  WaveSmem w[kWaves];
};

#ifdef MHQ_DIAG_STAMPS  // diagnostic build: cycles per phase, summed over waves
__device__ unsigned long long g_diag[8];
#define STAMP(i)                                                \
  do {                                                          \
    const unsigned long long _t = __builtin_amdgcn_s_memtime(); \
    ph[i] += _t - t_last;                                       \
    t_last = _t;                                                \
  } while (0)
#else
#define STAMP(i) \
  do {           \
  } while (0)
#endif

// One literal, one lane, straight from global memory: literals too large for a
// wave's LDS slice.  Same decision rules as the staged loop.
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

// Logical input word k of the staged tile.
__device__ __forceinline__ uint32_t in_word(const WaveSmem &ws, uint32_t k) { return ws.in_w[kInWords - 1u - k]; }

// One decode stream: decodes its list of literals one after the other.
struct Stream {
  uint64_t bb;      // next stream bits, MSB-aligned; nb >= 32 valid at every probe
  uint32_t nb;      // valid bits in bb
  uint32_t wi;      // logical index of the next word to append (= (p + nb) / 32)
  uint32_t nxt;     // that word, prefetched
  uint32_t p;       // bit position of bb's MSB
  uint32_t endbit;  // end of the current literal
  uint32_t optr;    // next output byte (staging byte index)
  uint32_t ostart;  // current literal's region start
  uint32_t oend;    // current literal's region end
  uint32_t acc;     // this stream's bytes of word optr>>2 below optr
  uint32_t bad;     // invalid code seen in the current literal
  uint32_t j;       // current literal (tile index) or kNone
  uint32_t i;       // position in this stream's rank list
  // per-iteration scratch
  uint32_t w0;
  uint64_t o64;
  bool fin;

  __device__ __forceinline__ bool active() const { return j != kNone; }

  // Starts literal lit (kNone: the stream is done).
  __device__ __forceinline__ void start(const WaveSmem &ws, uint32_t lit) {
    j = lit;
    acc = 0;
    if (lit == kNone) {  // done: keep every field harmless for the masked probes
      bb = 0;
      nb = 64;
      wi = 0;
      p = endbit = optr = ostart = oend = 0;
      bad = 0;
      return;
    }
    const uint2 r0 = ws.rec[lit], r1 = ws.rec[lit + 1];
    p = r0.x * 8u;
    endbit = r1.x * 8u;
    optr = ostart = r0.y;
    oend = r1.y;
    bad = 0;
#ifdef MHQ_DEC_BITBUF
    const uint32_t k = p >> 5, sh = p & 31u;
    const uint64_t pair = ((uint64_t)in_word(ws, k) << 32) | in_word(ws, k + 1);
    bb = pair << sh;
    nb = 64u - sh;
    wi = k + 2u;
    nxt = in_word(ws, wi);
#endif
  }
};

// Rank of the i-th literal of stream k ("snake": k, 2K-1-k, 2K+k, 4K-1-k, ...).
__device__ __forceinline__ uint32_t snake_rank(uint32_t k, uint32_t i) {
  return (i >> 1) * (2u * kK) + ((i & 1u) ? (2u * kK - 1u - k) : k);
}

__device__ __forceinline__ uint32_t next_literal_of(const WaveSmem &ws, uint32_t k, uint32_t i, uint32_t m) {
  const uint32_t r = snake_rank(k, i);
  return r < m ? (uint32_t)ws.order[r] : kNone;
}

struct Probe {
  uint32_t win, e, len0, tot, ns, syms;
};

#ifndef MHQ_DEC_BITBUF
// The 32 stream bits at bit position p (one ds_read2_b32 of logical words k, k+1).
__device__ __forceinline__ uint32_t window_at(const WaveSmem &ws, uint32_t p) {
  const uint32_t k = p >> 5, sh = p & 31u;
  const uint32_t *wp = ws.in_w + (kInWords - 2u - k);
  const uint64_t ww = (uint64_t)wp[0] | ((uint64_t)wp[1] << 32);  // {word k+1, word k}
  return (uint32_t)((ww << sh) >> 32);
}
#endif

__device__ __forceinline__ void probe_fast(Probe &q, const Stream &s, const WaveSmem &ws, const uint32_t *lut1) {
#ifdef MHQ_DEC_BITBUF
  q.win = (uint32_t)(s.bb >> 32);
#else
  q.win = window_at(ws, s.p);
#endif
  q.e = lut1[q.win >> (32 - kLut1Bits)];
  q.len0 = (q.e >> 16) & 31u;
  q.tot = (q.e >> 21) & 31u;
  q.ns = q.e >> 26;
  q.syms = q.e & 0xffffu;
}

// Codes of 13..30 bits, or the all-ones EOS prefix (rare in header text).
__device__ __forceinline__ void probe_long(Probe &q, Stream &s, const uint16_t *lut2) {
  const uint32_t rem = s.endbit - s.p;
  const uint32_t nw = ~q.win;
  const uint32_t c = nw ? (uint32_t)__builtin_clz(nw) : 32u;
  if (c >= (uint32_t)kEosOnes) {
    q.len0 = q.tot = 0xffffffffu;       // never fits: the literal ends here
    s.bad |= rem > (uint32_t)kEosOnes;  // a 31st bit exists: nil child
  } else {
    const uint32_t e2 = lut2[(c << kLut2SubBits) | ((q.win << (c + 1)) >> (32 - kLut2SubBits))];
    q.len0 = q.tot = (e2 >> 8) ? (e2 >> 8) : 0xffffffffu;
    q.ns = 1;
    q.syms = e2 & 0xffu;
  }
}

__device__ __forceinline__ void apply(const Probe &q, Stream &s, const WaveSmem &ws) {
  const uint32_t rem = s.endbit - s.p;
  const bool ct = q.tot <= rem;
  uint32_t cnt = ct ? q.ns : (q.len0 <= rem ? 1u : 0u);
  const uint32_t room = s.oend - s.optr;  // Read() stops once p is full (hc/huffman.go:104)
  cnt = cnt < room ? cnt : room;
  cnt = s.active() ? cnt : 0u;
  const uint32_t adv = cnt ? (ct ? q.tot : q.len0) : 0u;
  s.o64 |= (uint64_t)__builtin_amdgcn_ubfe(q.syms, 0, cnt * 8u) << ((s.optr - 4u * s.w0) * 8u);
  s.optr += cnt;
  s.fin |= cnt == 0;
#ifndef MHQ_DEC_BITBUF
  s.p += adv;
#else
  // consume adv bits, then top the buffer up to >= 32 bits from the prefetched word
  s.bb <<= adv;
  s.nb -= adv;
  s.p += adv;
  const bool need = s.nb <= 32u;
  s.bb |= need ? ((uint64_t)s.nxt << (32u - s.nb)) : 0ull;
  s.nb += need ? 32u : 0u;
  s.wi += need ? 1u : 0u;
  s.nxt = in_word(ws, s.wi);
#endif
}

__device__ __forceinline__ void flush(Stream &s, WaveSmem &ws) {
  if (s.o64) {
#ifdef MHQ_DIAG_PLAIN_OR  // diagnostic build: plain stores (wrong output), to price the atomics
    ws.out_w[s.w0] = (uint32_t)s.o64;
    ws.out_w[s.w0 + 1] = (uint32_t)(s.o64 >> 32);
#else
    atomicOr(&ws.out_w[s.w0], (uint32_t)s.o64);
    atomicOr(&ws.out_w[s.w0 + 1], (uint32_t)(s.o64 >> 32));
#endif
  }
  s.acc = (s.optr >> 2) != s.w0 ? (uint32_t)(s.o64 >> 32) : (uint32_t)s.o64;
}

// End of the current literal (EOF, full buffer or invalid code): record it and
// start the stream's next literal.
__device__ __forceinline__ void finish(Stream &s, WaveSmem &ws, uint32_t k, uint32_t m) {
  const uint32_t bad = s.optr != s.oend ? s.bad : 0u;
  ws.olen[s.j] = (s.optr - s.ostart) | (bad << 31);
  s.i++;
  s.start(ws, next_literal_of(ws, k, s.i, m));
}

// Two probes for each of the lane's two streams, interleaved.
__device__ __forceinline__ void iter2(Stream &a, Stream &b, WaveSmem &ws, const uint32_t *lut1,
                                      const uint16_t *lut2, uint32_t ka, uint32_t kb, uint32_t m) {
  a.w0 = a.optr >> 2;
  b.w0 = b.optr >> 2;
  a.o64 = a.acc;
  b.o64 = b.acc;
  a.fin = b.fin = false;
#pragma unroll
  for (int u = 0; u < 2; u++) {
    Probe qa, qb;
    probe_fast(qa, a, ws, lut1);
    probe_fast(qb, b, ws, lut1);
#ifndef MHQ_DIAG_NO_LONG
    if (qa.ns == 0) probe_long(qa, a, lut2);
    if (qb.ns == 0) probe_long(qb, b, lut2);
#endif
    apply(qa, a, ws);
    apply(qb, b, ws);
  }
  flush(a, ws);
  flush(b, ws);
  if (a.fin && a.active()) finish(a, ws, ka, m);
  if (b.fin && b.active()) finish(b, ws, kb, m);
}

// Two probes for one stream (kStreams == 1).
__device__ __forceinline__ void iter1(Stream &a, WaveSmem &ws, const uint32_t *lut1, const uint16_t *lut2,
                                      uint32_t ka, uint32_t m) {
  a.w0 = a.optr >> 2;
  a.o64 = a.acc;
  a.fin = false;
#pragma unroll
  for (int u = 0; u < 2; u++) {
    Probe qa;
    probe_fast(qa, a, ws, lut1);
    if (qa.ns == 0) probe_long(qa, a, lut2);
    apply(qa, a, ws);
  }
  flush(a, ws);
  if (a.fin && a.active()) finish(a, ws, ka, m);
}

// Counting sort of literals [0, m) by encoded length (bucketed) into ws.order.
__device__ __forceinline__ void order_by_length(WaveSmem &ws, uint32_t m, int lane) {
  ws.hist[lane] = 0;
  wave_sync();
  uint32_t bk[kPer], rk[kPer];
#pragma unroll
  for (int q = 0; q < kPer; q++) {
    const uint32_t j = (uint32_t)lane + (uint32_t)q * kWave;
    bk[q] = 0;
    rk[q] = 0;
    if (j < m) {
      const uint32_t bytes = ws.rec[j + 1].x - ws.rec[j].x;
      bk[q] = bytes < 32u ? bytes : min(32u + ((bytes - 32u) >> 4), (uint32_t)kBuckets - 1u);
      rk[q] = atomicAdd(&ws.hist[bk[q]], 1u);
    }
  }
  wave_sync();
  // exclusive scan of the 64 bucket counts (lane b holds bucket b)
  const uint32_t h = ws.hist[lane];
  uint32_t x = h;
#pragma unroll
  for (int d = 1; d < kWave; d <<= 1) {
    const uint32_t y = __shfl_up(x, d);
    if (lane >= d) x += y;
  }
  ws.hist[lane] = x - h;
  wave_sync();
#pragma unroll
  for (int q = 0; q < kPer; q++) {
    const uint32_t j = (uint32_t)lane + (uint32_t)q * kWave;
    if (j < m) ws.order[ws.hist[bk[q]] + rk[q]] = (uint16_t)j;
  }
  wave_sync();
}

__global__ __launch_bounds__(kThreads) void decode_kernel(
    const uint8_t *__restrict__ in, const uint64_t *__restrict__ in_off, uint64_t in_bias, uint64_t n,
    uint8_t *__restrict__ out, const uint64_t *__restrict__ out_off, uint64_t out_bias,
    uint32_t *__restrict__ out_len, uint8_t *__restrict__ status, const uint32_t *__restrict__ g_lut1,
    const uint16_t *__restrict__ g_lut2, uint64_t ntiles) {
  __shared__ Smem sm;
  const int tid = threadIdx.x;
  const int wave = __builtin_amdgcn_readfirstlane(tid / kWave);
  const int lane = tid % kWave;
  for (int i = tid; i < kLut1Size / 4; i += kThreads) ((u32x4 *)sm.lut1)[i] = ((const u32x4 *)g_lut1)[i];
  for (int i = tid; i < kLut2Size / 8; i += kThreads) ((u32x4 *)sm.lut2)[i] = ((const u32x4 *)g_lut2)[i];
  __syncthreads();

  WaveSmem &ws = sm.w[wave];
  const uint32_t *lut1 = sm.lut1;
  const uint16_t *lut2 = sm.lut2;
  const uint64_t stride = (uint64_t)gridDim.x * kWaves;
#ifdef MHQ_DIAG_STAMPS
  unsigned long long ph[6] = {0, 0, 0, 0, 0, 0};
  unsigned long long t_last = __builtin_amdgcn_s_memtime();
#endif

  for (uint64_t t = (uint64_t)blockIdx.x * kWaves + wave; t < ntiles; t += stride) {
    const uint64_t s = t * kTileLits;
    const uint32_t cnt = (uint32_t)min((uint64_t)kTileLits, n - s);
    TileOffsets<kTileLits> off;
    off.load(in_off, out_off, s, cnt, lane);

    uint32_t cur = 0;
    while (cur < cnt) {
      const uint64_t ic = in_off[s + cur], oc = out_off[s + cur];  // wave-uniform
      const uint8_t *ia = in + (ic - in_bias);
      uint8_t *oa = out + (oc - out_bias);
      const uint32_t idelta = (uint32_t)((uintptr_t)ia & 15u);
      const uint32_t odelta = (uint32_t)((uintptr_t)oa & 15u);
      const uint32_t end = off.fit(cur, cnt, ic, kInCap - idelta, oc, kOutCap - odelta, lane);
      STAMP(0);
      if (end == cur) {  // one literal larger than the slice
        if (lane == 0)
          decode_literal_global(ia, in_off[s + cur + 1] - ic, oa, out_off[s + cur + 1] - oc, lut1, lut2,
                                out_len + s + cur, status + s + cur);
        cur++;
        continue;
      }
      const uint32_t m = end - cur;
#pragma unroll
      for (int k = 0; k < TileOffsets<kTileLits>::kPer; k++) {
        const uint32_t j = (uint32_t)lane + (uint32_t)k * kWave;
        if (j >= cur && j <= end)
          ws.rec[j - cur] = make_uint2((uint32_t)(off.io[k] - ic) + idelta, (uint32_t)(off.oo[k] - oc) + odelta);
      }
      const uint32_t in_bytes = (uint32_t)(in_off[s + end] - ic) + idelta;
      const uint32_t out_bytes = (uint32_t)(out_off[s + end] - oc) + odelta;
      stage_in<true, true>(ws.in_w, kInWords, ia - idelta, in_bytes, lane);
      zero_lds(ws.out_w, out_bytes, lane);
      wave_sync();
      STAMP(1);

      order_by_length(ws, m, lane);
      const uint32_t ka = (uint32_t)lane, kb = (uint32_t)lane + kWave;
      Stream a, b;
      a.i = 0;
      b.i = 0;
      a.start(ws, next_literal_of(ws, ka, 0, m));
      if (kStreams == 2) b.start(ws, next_literal_of(ws, kb, 0, m));
      else b.start(ws, kNone);
#ifdef MHQ_DIAG_ONE_STREAM  // diagnostic build: only stream a works (wrong output)
      b.start(ws, kNone);
#endif
#ifdef MHQ_DIAG_NO_DECODE  // diagnostic build: staging and stores only
      a.j = b.j = kNone;
#endif
      STAMP(2);
      while (a.active() || b.active()) {
        if (kStreams == 2) iter2(a, b, ws, lut1, lut2, ka, kb, m);
        else iter1(a, ws, lut1, lut2, ka, m);
#ifdef MHQ_DIAG_STAMPS
        ph[5]++;
#endif
      }
      wave_sync();
      STAMP(3);
      store_out(oa - odelta, (const uint8_t *)ws.out_w, odelta, out_bytes, lane);
      for (uint32_t i = lane; i < m; i += kWave) {
        const uint32_t v = ws.olen[i];
        out_len[s + cur + i] = v & 0x7fffffffu;
        status[s + cur + i] = (uint8_t)(v >> 31);
      }
      wave_sync();
      STAMP(4);
      cur = end;
    }
  }
#ifdef MHQ_DIAG_STAMPS
  if (lane == 0)
    for (int i = 0; i < 6; i++) atomicAdd(&g_diag[i], ph[i]);
#endif
}

}  // namespace

#ifdef MHQ_DIAG_STAMPS
extern "C" int mhq_diag_read(unsigned long long *out, int n) {
  unsigned long long h[8];
  if (hipMemcpyFromSymbol(h, HIP_SYMBOL(g_diag), sizeof(h)) != hipSuccess) return -1;
  for (int i = 0; i < n && i < 8; i++) out[i] = h[i];
  unsigned long long z[8] = {0};
  return hipMemcpyToSymbol(HIP_SYMBOL(g_diag), z, sizeof(z)) == hipSuccess ? 0 : -1;
}
#endif

hipError_t launch_decode(const DevTables &t, const uint8_t *in, const uint64_t *in_off, uint64_t in_bias,
                         uint64_t n, uint8_t *out, const uint64_t *out_off, uint64_t out_bias,
                         uint32_t *out_len, uint8_t *status, hipStream_t s) {
  if (n == 0) return hipSuccess;
  const uint64_t ntiles = (n + kTileLits - 1) / kTileLits;
  decode_kernel<<<dim3(dev::tile_grid(ntiles, kWaves, 1)), dim3(kThreads), 0, s>>>(
      in, in_off, in_bias, n, out, out_off, out_bias, out_len, status, t.lut1, t.lut2, ntiles);
  return hipGetLastError();
}

}  // namespace mhq
