// huff_kernels.hip -- gfx950 (CDNA4) kernels for the RFC 7541 Huffman literal
// batch codec.  Bit-exact with minhq's hc/huffman.go + io/bitio.go (semantics
// contract: SURVEY.md §8a; restated in oracle/huff_oracle.c).
//
// Work decomposition (all three codec kernels):
//   * a workgroup is kWaves wave64s sharing the code tables in LDS; every wave
//     independently walks tiles of kTileLits consecutive literals;
//   * a tile is staged through LDS: its offsets (coalesced u64 loads), its
//     input bytes (coalesced 16-B loads; decode input is stored byte-swapped
//     so bit 31 of a word is the first stream bit), and for decode/encode the
//     whole output region, zero-filled, in global layout, written back with
//     aligned 16-B stores;
//   * if a tile does not fit the wave's LDS slice it is processed as several
//     sub-tiles (maximal prefixes that fit); a single literal too large for
//     the slice is handled by one lane straight from global memory;
//   * inside a (sub-)tile each lane owns a contiguous run of literals holding
//     ~1/64 of the tile's input bytes (lower_bound per lane) and streams it
//     with one flat loop: literal boundaries are a branch inside the loop, not
//     a loop nest, so lanes never wait for each other's literals.
//
// Decode probes LUT1 (4096 x u32, up to two symbols per 12-bit probe) and, for
// codes of 13..30 bits, LUT2 keyed by the count of leading ones (huff_table.h).
#include <hip/hip_runtime.h>

#include "huff_kernels.h"
#include "huff_table.h"

namespace mhq {

namespace {

constexpr int kWave = 64;
typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));

__device__ __forceinline__ void wave_sync() {
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

__device__ __forceinline__ uint32_t popc64(uint64_t m) { return (uint32_t)__popcll(m); }

// ---------------------------------------------------------------------------
// Tile plumbing shared by the kernels.
// ---------------------------------------------------------------------------
template <int kTileLits>
struct TileOffsets {
  static constexpr int kPer = (kTileLits + 1 + kWave - 1) / kWave;
  uint64_t io[kPer];  // in_off[s + lane + 64k]
  uint64_t oo[kPer];  // out_off[s + lane + 64k] (unused by encode_len)

  __device__ __forceinline__ void load(const uint64_t *__restrict__ in_off, const uint64_t *__restrict__ out_off,
                                       uint64_t s, uint32_t cnt, int lane) {
#pragma unroll
    for (int k = 0; k < kPer; k++) {
      const uint32_t j = (uint32_t)lane + (uint32_t)k * kWave;
      io[k] = j <= cnt ? __builtin_nontemporal_load(in_off + s + j) : 0;
      oo[k] = (out_off && j <= cnt) ? __builtin_nontemporal_load(out_off + s + j) : 0;
    }
  }

  // Literals [cur, end] fit when their input span (from the 16-B aligned start)
  // is <= in_lim and their output span <= out_lim.  Returns end (>= cur; == cur
  // means literal `cur` alone does not fit).
  __device__ __forceinline__ uint32_t fit(uint32_t cur, uint32_t cnt, uint64_t in_lo, uint64_t in_lim,
                                          uint64_t out_lo, uint64_t out_lim, int lane) const {
    uint32_t n = 0;
#pragma unroll
    for (int k = 0; k < kPer; k++) {
      const uint32_t j = (uint32_t)lane + (uint32_t)k * kWave;
      const bool ok = j > cur && j <= cnt && (io[k] - in_lo) <= in_lim && (oo[k] - out_lo) <= out_lim;
      n += popc64(__ballot(ok));
    }
    return cur + n;
  }
};

// First index i in [0, m) with key(i) >= target, or m.
template <class K>
__device__ __forceinline__ uint32_t lower_bound(K key, uint32_t m, uint32_t target) {
  uint32_t lo = 0, hi = m;
  while (lo < hi) {
    const uint32_t mid = (lo + hi) >> 1;
    if (key(mid) < target) lo = mid + 1;
    else hi = mid;
  }
  return lo;
}

// Byte-balanced split of literals [0, m) (input byte starts key(i)) into 64
// contiguous runs.
template <class K>
__device__ __forceinline__ void lane_run(K key, uint32_t m, int lane, uint32_t &first, uint32_t &last) {
  const uint32_t b0 = key(0);
  const uint32_t total = key(m) - b0;
  const uint32_t t0 = b0 + (uint32_t)(((uint64_t)total * (uint32_t)lane) >> 6);
  const uint32_t t1 = b0 + (uint32_t)(((uint64_t)total * (uint32_t)(lane + 1)) >> 6);
  first = lane == 0 ? 0u : lower_bound(key, m, t0);
  last = lane == kWave - 1 ? m : lower_bound(key, m, t1);
}

// Copies global bytes [a, a+nbytes) (a 16-B aligned address) into LDS words.
template <bool kSwap>
__device__ __forceinline__ void stage_in(uint32_t *lds, const uint8_t *a, uint32_t nbytes, int lane) {
  const uint32_t chunks = (nbytes + 15u) >> 4;
  const u32x4 *src = (const u32x4 *)a;
  for (uint32_t c = lane; c < chunks; c += kWave) {
    u32x4 v = __builtin_nontemporal_load(src + c);  // an aligned chunk holding a valid byte never crosses a page
    if (kSwap) {
      v.x = __builtin_bswap32(v.x);
      v.y = __builtin_bswap32(v.y);
      v.z = __builtin_bswap32(v.z);
      v.w = __builtin_bswap32(v.w);
    }
    *(u32x4 *)(lds + 4 * c) = v;
  }
}

__device__ __forceinline__ void zero_lds(uint8_t *lds, uint32_t nbytes, int lane) {
  const uint32_t chunks = (nbytes + 15u) >> 4;
  for (uint32_t c = lane; c < chunks; c += kWave) *(uint4 *)(lds + 16 * c) = make_uint4(0, 0, 0, 0);
}

// Writes LDS bytes [lo, hi) to global o_al + [lo, hi), o_al 16-B aligned.
// Whole 16-B chunks go out as one aligned store; the (at most two) partial
// chunks at the ends are written byte by byte so neighbours are untouched.
__device__ __forceinline__ void store_out(uint8_t *o_al, const uint8_t *lds, uint32_t lo, uint32_t hi, int lane) {
  if (hi <= lo) return;
  const uint32_t c0 = lo >> 4, c1 = (hi + 15u) >> 4;
  for (uint32_t c = c0 + lane; c < c1; c += kWave) {
    const uint32_t a = c << 4, b = a + 16u;
    if (a >= lo && b <= hi) {
      __builtin_nontemporal_store(*(const u32x4 *)(lds + a), (u32x4 *)(o_al + a));
    } else {
      const uint32_t x0 = a > lo ? a : lo, x1 = b < hi ? b : hi;
      for (uint32_t x = x0; x < x1; x++) o_al[x] = lds[x];
    }
  }
}

// ---------------------------------------------------------------------------
// Decode (hc/huffman.go:102-121 + the ReadFull loop, hc/io.go:85-96).
// ---------------------------------------------------------------------------
namespace dec {
constexpr int kWaves = 8;
constexpr int kThreads = kWave * kWaves;
constexpr int kTileLits = 256;
constexpr int kInCap = 6144;   // staged input bytes per wave (incl. 16-B alignment slack)
constexpr int kOutCap = 8192;  // staged output bytes per wave

struct WaveSmem {
  uint32_t in_w[kInCap / 4 + 4];  // byte-swapped input words (+ tail for window reads)
  uint8_t out_b[kOutCap + 16];    // output staging (+ one spare word pair)
  uint2 rec[kTileLits + 2];       // per boundary: (input byte index, output byte index)
  uint32_t olen[kTileLits];       // out_len | status << 31
};
struct Smem {
  uint32_t lut1[kLut1Size];
  uint16_t lut2[kLut2Size];
  WaveSmem w[kWaves];
};
}  // namespace dec

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

__global__ __launch_bounds__(dec::kThreads) void decode_kernel(
    const uint8_t *__restrict__ in, const uint64_t *__restrict__ in_off, uint64_t in_bias, uint64_t n,
    uint8_t *__restrict__ out, const uint64_t *__restrict__ out_off, uint64_t out_bias,
    uint32_t *__restrict__ out_len, uint8_t *__restrict__ status, const uint32_t *__restrict__ g_lut1,
    const uint16_t *__restrict__ g_lut2, uint64_t ntiles) {
  using namespace dec;
  __shared__ Smem sm;
  const int tid = threadIdx.x;
  const int wave = __builtin_amdgcn_readfirstlane(tid / kWave);
  const int lane = tid % kWave;
  for (int i = tid; i < kLut1Size / 4; i += kThreads) ((uint4 *)sm.lut1)[i] = ((const uint4 *)g_lut1)[i];
  for (int i = tid; i < kLut2Size / 8; i += kThreads) ((uint4 *)sm.lut2)[i] = ((const uint4 *)g_lut2)[i];
  __syncthreads();

  WaveSmem &ws = sm.w[wave];
  const uint32_t *lut1 = sm.lut1;
  const uint16_t *lut2 = sm.lut2;
  const uint64_t stride = (uint64_t)gridDim.x * kWaves;

  for (uint64_t t = (uint64_t)blockIdx.x * kWaves + wave; t < ntiles; t += stride) {
    const uint64_t s = t * kTileLits;
    const uint32_t cnt = (uint32_t)min((uint64_t)kTileLits, n - s);
    TileOffsets<kTileLits> off;
    off.load(in_off, out_off, s, cnt, lane);

    uint32_t cur = 0;
    while (cur < cnt) {
      const uint64_t ic = in_off[s + cur], oc = out_off[s + cur];  // wave-uniform (scalar loads)
      const uint8_t *ia = in + (ic - in_bias);
      uint8_t *oa = out + (oc - out_bias);
      const uint32_t idelta = (uint32_t)((uintptr_t)ia & 15u);
      const uint32_t odelta = (uint32_t)((uintptr_t)oa & 15u);
      const uint32_t end = off.fit(cur, cnt, ic, kInCap - idelta, oc, kOutCap - odelta, lane);
      if (end == cur) {  // one literal larger than the slice
        if (lane == 0)
          decode_literal_global(ia, in_off[s + cur + 1] - ic, oa, out_off[s + cur + 1] - oc, lut1, lut2,
                                out_len + s + cur, status + s + cur);
        cur++;
        continue;
      }
      const uint32_t m = end - cur;
      // boundary records relative to the staged slices
#pragma unroll
      for (int k = 0; k < TileOffsets<kTileLits>::kPer; k++) {
        const uint32_t j = (uint32_t)lane + (uint32_t)k * kWave;
        if (j >= cur && j <= end)
          ws.rec[j - cur] = make_uint2((uint32_t)(off.io[k] - ic) + idelta, (uint32_t)(off.oo[k] - oc) + odelta);
      }
      const uint32_t in_bytes = (uint32_t)(in_off[s + end] - ic) + idelta;
      const uint32_t out_bytes = (uint32_t)(out_off[s + end] - oc) + odelta;
      stage_in<true>(ws.in_w, ia - idelta, in_bytes, lane);
      zero_lds(ws.out_b, out_bytes, lane);
      wave_sync();

      uint32_t j, last;
      lane_run([&](uint32_t i) { return ws.rec[i].x; }, m, lane, j, last);
#ifdef MHQ_DIAG_NO_DECODE  // diagnostic build: staging and stores only
      for (uint32_t i = j; i < last; i++) ws.olen[i] = ws.rec[i + 1].y - ws.rec[i].y;
      j = last;
#endif
      if (j < last) {
        // Lane state.  Output bytes are packed into registers on the LDS word
        // grid and OR-ed into the zeroed staging words: a lane only ever ORs
        // its own bytes (zeros elsewhere), so words shared with a neighbouring
        // lane at run boundaries need no ordering.
        uint32_t p = ws.rec[j].x * 8u;  // next code's bit position
        uint2 r = ws.rec[j + 1];
        uint32_t endbit = r.x * 8u;     // end of this literal
        uint32_t optr = ws.rec[j].y, ostart = optr, oend = r.y;
        uint32_t acc = 0;               // this lane's bytes of word optr>>2 below optr
        uint32_t bad = 0;
        uint32_t *ow = (uint32_t *)ws.out_b;
        while (j < last) {
          const uint32_t w0 = optr >> 2;
          uint64_t o64 = acc;
          bool fin = false;
#pragma unroll
          for (int u = 0; u < 2; u++) {  // two probes per iteration, one output flush
            const uint32_t k = p >> 5, sh = p & 31u;
            const uint64_t ww = ((uint64_t)ws.in_w[k] << 32) | ws.in_w[k + 1];
            const uint32_t win = (uint32_t)((ww << sh) >> 32);
            const uint32_t e = lut1[win >> (32 - kLut1Bits)];
            const uint32_t rem = endbit - p;
            uint32_t len0 = (e >> 16) & 31u, tot = (e >> 21) & 31u, ns = e >> 26, syms = e & 0xffffu;
            if (ns == 0) {  // a code of 13..30 bits, or the all-ones EOS prefix
              const uint32_t nw = ~win;
              const uint32_t c = nw ? (uint32_t)__builtin_clz(nw) : 32u;
              if (c >= (uint32_t)kEosOnes) {
                len0 = tot = 0xffffffffu;       // never fits: the literal ends here
                bad |= rem > (uint32_t)kEosOnes;  // a 31st bit exists: nil child
              } else {
                const uint32_t e2 = lut2[(c << kLut2SubBits) | ((win << (c + 1)) >> (32 - kLut2SubBits))];
                len0 = tot = (e2 >> 8) ? (e2 >> 8) : 0xffffffffu;
                ns = 1;
                syms = e2 & 0xffu;
              }
            }
            const bool ct = tot <= rem;
            uint32_t cnt = ct ? ns : (len0 <= rem ? 1u : 0u);
            const uint32_t adv = ct ? tot : len0;
            const uint32_t room = oend - optr;  // Read() stops once p is full (hc/huffman.go:104)
            cnt = cnt < room ? cnt : room;
            o64 |= (uint64_t)__builtin_amdgcn_ubfe(syms, 0, cnt * 8u) << ((optr - 4u * w0) * 8u);
            optr += cnt;
            p += cnt ? adv : 0u;
            fin |= cnt == 0;
          }
          atomicOr(&ow[w0], (uint32_t)o64);
          atomicOr(&ow[w0 + 1], (uint32_t)(o64 >> 32));
          acc = (optr >> 2) != w0 ? (uint32_t)(o64 >> 32) : (uint32_t)o64;
          if (fin) {  // end of this literal (EOF, full buffer or invalid code)
            bad = optr != oend ? bad : 0u;
            ws.olen[j] = (optr - ostart) | (bad << 31);
            j++;
            bad = 0;
            r = ws.rec[j + 1];
            p = endbit;
            endbit = r.x * 8u;
            if ((oend >> 2) != (optr >> 2)) acc = 0;  // bytes below the next region are slack
            optr = ostart = oend;
            oend = r.y;
          }
        }
      }
      wave_sync();
      store_out(oa - odelta, ws.out_b, odelta, out_bytes, lane);
      for (uint32_t i = lane; i < m; i += kWave) {
        const uint32_t v = ws.olen[i];
        out_len[s + cur + i] = v & 0x7fffffffu;
        status[s + cur + i] = (uint8_t)(v >> 31);
      }
      wave_sync();
      cur = end;
    }
  }
}

// ---------------------------------------------------------------------------
// Encode length (hc/huffman.go:23-37 sizing; the Auto input, hc/io.go:172).
// ---------------------------------------------------------------------------
namespace enc {
constexpr int kWaves = 8;
constexpr int kThreads = kWave * kWaves;
constexpr int kTileLits = 256;
constexpr int kInCap = 8192;
constexpr int kOutCap = 8192;

struct LenWaveSmem {
  uint32_t in_w[kInCap / 4 + 4];
  uint32_t rec[kTileLits + 1];
};
struct LenSmem {
  uint32_t len[256];
  LenWaveSmem w[kWaves];
};
struct WaveSmem {
  uint32_t in_w[kInCap / 4 + 4];
  uint32_t out_w[kOutCap / 4 + 4];
  uint2 rec[kTileLits + 1];
};
struct Smem {
  uint2 code[256];  // (code left-aligned in 32 bits, length)
  WaveSmem w[kWaves];
};
}  // namespace enc

__device__ __forceinline__ uint32_t lds_byte(const uint32_t *w, uint32_t x) {
  return (w[x >> 2] >> ((x & 3u) * 8u)) & 0xffu;
}

__global__ __launch_bounds__(enc::kThreads) void encode_len_kernel(
    const uint8_t *__restrict__ in, const uint64_t *__restrict__ in_off, uint64_t in_bias, uint64_t n,
    uint32_t *__restrict__ enc_len, const uint8_t *__restrict__ g_len, uint64_t ntiles) {
  using namespace enc;
  __shared__ LenSmem sm;
  const int tid = threadIdx.x;
  const int wave = __builtin_amdgcn_readfirstlane(tid / kWave);
  const int lane = tid % kWave;
  for (int i = tid; i < 256; i += kThreads) sm.len[i] = g_len[i];
  __syncthreads();
  LenWaveSmem &ws = sm.w[wave];
  const uint64_t stride = (uint64_t)gridDim.x * kWaves;
  for (uint64_t t = (uint64_t)blockIdx.x * kWaves + wave; t < ntiles; t += stride) {
    const uint64_t s = t * kTileLits;
    const uint32_t cnt = (uint32_t)min((uint64_t)kTileLits, n - s);
    TileOffsets<kTileLits> off;
    off.load(in_off, nullptr, s, cnt, lane);
    uint32_t cur = 0;
    while (cur < cnt) {
      const uint64_t ic = in_off[s + cur];
      const uint8_t *ia = in + (ic - in_bias);
      const uint32_t idelta = (uint32_t)((uintptr_t)ia & 15u);
      const uint32_t end = off.fit(cur, cnt, ic, kInCap - idelta, 0, ~0ull, lane);
      if (end == cur) {  // one huge literal: this lane sums it from global memory
        if (lane == 0) {
          const uint64_t L = in_off[s + cur + 1] - ic;
          uint64_t bits = 0;
          for (uint64_t i = 0; i < L; i++) bits += sm.len[ia[i]];
          enc_len[s + cur] = (uint32_t)((bits + 7u) >> 3);
        }
        cur++;
        continue;
      }
      const uint32_t m = end - cur;
#pragma unroll
      for (int k = 0; k < TileOffsets<kTileLits>::kPer; k++) {
        const uint32_t j = (uint32_t)lane + (uint32_t)k * kWave;
        if (j >= cur && j <= end) ws.rec[j - cur] = (uint32_t)(off.io[k] - ic) + idelta;
      }
      const uint32_t in_bytes = (uint32_t)(in_off[s + end] - ic) + idelta;
      stage_in<false>(ws.in_w, ia - idelta, in_bytes, lane);
      wave_sync();
      uint32_t j, last;
      lane_run([&](uint32_t i) { return ws.rec[i]; }, m, lane, j, last);
      if (j < last) {
        uint32_t x = ws.rec[j], xend = ws.rec[j + 1];
        uint32_t bits = 0;
        while (true) {
          if (x < xend) {
            // whole aligned words where possible
            if ((x & 3u) == 0 && x + 4 <= xend) {
              const uint32_t w = ws.in_w[x >> 2];
              bits += sm.len[w & 0xffu] + sm.len[(w >> 8) & 0xffu] + sm.len[(w >> 16) & 0xffu] + sm.len[w >> 24];
              x += 4;
            } else {
              bits += sm.len[lds_byte(ws.in_w, x)];
              x++;
            }
          } else {
            enc_len[s + cur + j] = (bits + 7u) >> 3;
            if (++j >= last) break;
            bits = 0;
            xend = ws.rec[j + 1];
          }
        }
      }
      wave_sync();
      cur = end;
    }
  }
}

// ---------------------------------------------------------------------------
// Encode (hc/huffman.go:23-37 over io/bitio.go:72-149): codes MSB-first, the
// last octet padded with 1 bits.  Output words are assembled in registers on
// the LDS word grid and OR-ed into the zeroed staging area (a word may be
// shared by two lanes at run boundaries, hence the OR).
// ---------------------------------------------------------------------------
__global__ __launch_bounds__(enc::kThreads) void encode_kernel(
    const uint8_t *__restrict__ in, const uint64_t *__restrict__ in_off, uint64_t in_bias, uint64_t n,
    uint8_t *__restrict__ out, const uint64_t *__restrict__ out_off, uint64_t out_bias,
    const uint32_t *__restrict__ g_code, const uint8_t *__restrict__ g_len, uint64_t ntiles) {
  using namespace enc;
  __shared__ Smem sm;
  const int tid = threadIdx.x;
  const int wave = __builtin_amdgcn_readfirstlane(tid / kWave);
  const int lane = tid % kWave;
  for (int i = tid; i < 256; i += kThreads) {
    const uint32_t L = g_len[i];
    sm.code[i] = make_uint2(g_code[i] << (32u - L), L);
  }
  __syncthreads();
  WaveSmem &ws = sm.w[wave];
  const uint64_t stride = (uint64_t)gridDim.x * kWaves;
  for (uint64_t t = (uint64_t)blockIdx.x * kWaves + wave; t < ntiles; t += stride) {
    const uint64_t s = t * kTileLits;
    const uint32_t cnt = (uint32_t)min((uint64_t)kTileLits, n - s);
    TileOffsets<kTileLits> off;
    off.load(in_off, out_off, s, cnt, lane);
    uint32_t cur = 0;
    while (cur < cnt) {
      const uint64_t ic = in_off[s + cur], oc = out_off[s + cur];
      const uint8_t *ia = in + (ic - in_bias);
      uint8_t *oa = out + (oc - out_bias);
      const uint32_t idelta = (uint32_t)((uintptr_t)ia & 15u);
      const uint32_t odelta = (uint32_t)((uintptr_t)oa & 15u);
      const uint32_t end = off.fit(cur, cnt, ic, kInCap - idelta, oc, kOutCap - odelta, lane);
      if (end == cur) {  // one huge literal: lane 0 encodes it byte-serially to global memory
        if (lane == 0) {
          const uint64_t L = in_off[s + cur + 1] - ic, cap = out_off[s + cur + 1] - oc;
          uint64_t acc = 0, o = 0;
          uint32_t nacc = 0;
          for (uint64_t i = 0; i < L; i++) {
            const uint2 cl = sm.code[ia[i]];
            acc = (acc << cl.y) | (cl.x >> (32u - cl.y));
            nacc += cl.y;
            while (nacc >= 8) {
              nacc -= 8;
              if (o < cap) oa[o] = (uint8_t)(acc >> nacc);
              o++;
            }
          }
          if (nacc && o < cap) oa[o] = (uint8_t)((acc << (8 - nacc)) | ((1u << (8 - nacc)) - 1u));
        }
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
      stage_in<false>(ws.in_w, ia - idelta, in_bytes, lane);
      zero_lds((uint8_t *)ws.out_w, out_bytes, lane);
      wave_sync();
      uint32_t j, last;
      lane_run([&](uint32_t i) { return ws.rec[i].x; }, m, lane, j, last);
      if (j < last) {
        uint2 r0 = ws.rec[j], r1 = ws.rec[j + 1];
        uint32_t x = r0.x, xend = r1.x;
        uint32_t bp = r0.y * 8u;            // absolute output bit position in the staging words
        uint32_t obits_end = r1.y * 8u;     // end of this literal's region
        uint64_t acc = 0;                   // bits of word bp>>5 onwards, MSB-aligned at bit 63
        uint32_t *ow = ws.out_w;
        while (true) {
          if (x < xend) {
            const uint2 cl = sm.code[lds_byte(ws.in_w, x)];
            x++;
            const uint32_t sh = bp & 31u;
            acc |= ((uint64_t)cl.x << 32) >> sh;
            bp += cl.y;
            if (sh + cl.y >= 32u) {  // the word at the old position is complete
              if (bp - cl.y < obits_end) atomicOr(&ow[(bp - cl.y) >> 5], __builtin_bswap32((uint32_t)(acc >> 32)));
              acc <<= 32;
            }
          } else {
            // Pad(0xff): fill to the octet boundary with 1 bits, then flush the partial word
            const uint32_t pad = (8u - (bp & 7u)) & 7u;
            const uint32_t sh = bp & 31u;
            if (pad) acc |= ((((uint64_t)1 << pad) - 1u) << (64u - pad)) >> sh;
            bp += pad;
            if ((bp & 31u) != 0 || pad) {
              const uint32_t wpos = (bp - 1u) >> 5;  // the word holding the last written bit
              if (bp <= obits_end && ((bp & 31u) != 0 || sh != 0 || pad))
                atomicOr(&ow[wpos], __builtin_bswap32((uint32_t)(acc >> 32)));
            }
            if (++j >= last) break;
            r1 = ws.rec[j + 1];
            x = xend;
            xend = r1.x;
            bp = obits_end;  // the next region starts where this one ends
            obits_end = r1.y * 8u;
            acc = 0;
          }
        }
      }
      wave_sync();
      store_out(oa - odelta, (const uint8_t *)ws.out_w, odelta, out_bytes, lane);
      wave_sync();
      cur = end;
    }
  }
}

// ---------------------------------------------------------------------------
// Exclusive scans for offsets (three passes: block sums, scan of sums, apply).
// ---------------------------------------------------------------------------
constexpr int kScanBlock = 256;
constexpr int kScanItems = 8;
constexpr int kScanChunk = kScanBlock * kScanItems;

struct LenVal {  // enc_len -> (bytes, decode capacity)
  const uint32_t *len;
  __device__ inline void operator()(uint64_t i, uint64_t &a, uint64_t &b) const {
    const uint64_t v = len[i];
    a = v;
    b = (v * 8u) / 5u;
  }
};
struct CapVal {  // in_off -> decode capacity floor(8*len/5)
  const uint64_t *off;
  __device__ inline void operator()(uint64_t i, uint64_t &a, uint64_t &b) const {
    const uint64_t v = off[i + 1] - off[i];
    a = (v * 8u) / 5u;
    b = 0;
  }
};

__device__ inline void block_scan2(uint64_t &a, uint64_t &b, uint64_t *sa, uint64_t *sb, uint64_t &ta,
                                   uint64_t &tb) {
  // inclusive scan of (a,b) across the block; returns block totals
  const int tid = threadIdx.x;
  sa[tid] = a;
  sb[tid] = b;
  __syncthreads();
  for (int d = 1; d < kScanBlock; d <<= 1) {
    uint64_t xa = 0, xb = 0;
    if (tid >= d) {
      xa = sa[tid - d];
      xb = sb[tid - d];
    }
    __syncthreads();
    sa[tid] += xa;
    sb[tid] += xb;
    __syncthreads();
  }
  a = sa[tid];
  b = sb[tid];
  ta = sa[kScanBlock - 1];
  tb = sb[kScanBlock - 1];
  __syncthreads();
}

template <class F>
__global__ __launch_bounds__(kScanBlock) void scan_reduce_kernel(F f, uint64_t n, uint64_t *sums) {
  __shared__ uint64_t sa[kScanBlock], sb[kScanBlock];
  const uint64_t base = (uint64_t)blockIdx.x * kScanChunk + (uint64_t)threadIdx.x * kScanItems;
  uint64_t a = 0, b = 0;
  for (int k = 0; k < kScanItems; k++) {
    if (base + k < n) {
      uint64_t x, y;
      f(base + k, x, y);
      a += x;
      b += y;
    }
  }
  uint64_t ta, tb;
  block_scan2(a, b, sa, sb, ta, tb);
  if (threadIdx.x == 0) {
    sums[2 * blockIdx.x] = ta;
    sums[2 * blockIdx.x + 1] = tb;
  }
}

__global__ __launch_bounds__(kScanBlock) void scan_sums_kernel(uint64_t *sums, uint64_t nb) {
  __shared__ uint64_t sa[kScanBlock], sb[kScanBlock];
  uint64_t carry_a = 0, carry_b = 0;
  for (uint64_t base = 0; base < nb; base += kScanBlock) {
    const uint64_t i = base + threadIdx.x;
    uint64_t a = i < nb ? sums[2 * i] : 0, b = i < nb ? sums[2 * i + 1] : 0;
    const uint64_t ea = a, eb = b;
    uint64_t ta, tb;
    block_scan2(a, b, sa, sb, ta, tb);
    if (i < nb) {  // exclusive
      sums[2 * i] = carry_a + a - ea;
      sums[2 * i + 1] = carry_b + b - eb;
    }
    carry_a += ta;
    carry_b += tb;
  }
}

template <class F>
__global__ __launch_bounds__(kScanBlock) void scan_apply_kernel(F f, uint64_t n, const uint64_t *sums,
                                                                 uint64_t base_val, uint64_t *oa,
                                                                 uint64_t *ob) {
  __shared__ uint64_t sa[kScanBlock], sb[kScanBlock];
  const uint64_t base = (uint64_t)blockIdx.x * kScanChunk + (uint64_t)threadIdx.x * kScanItems;
  uint64_t xa[kScanItems], xb[kScanItems];
  uint64_t a = 0, b = 0;
#pragma unroll
  for (int k = 0; k < kScanItems; k++) {
    xa[k] = 0;
    xb[k] = 0;
    if (base + k < n) f(base + k, xa[k], xb[k]);
    a += xa[k];
    b += xb[k];
  }
  const uint64_t la = a, lb = b;
  uint64_t ta, tb;
  block_scan2(a, b, sa, sb, ta, tb);
  uint64_t ra = base_val + sums[2 * blockIdx.x] + a - la;
  uint64_t rb = base_val + sums[2 * blockIdx.x + 1] + b - lb;
#pragma unroll
  for (int k = 0; k < kScanItems; k++) {
    if (base + k <= n) {  // position n receives the grand total
      if (oa) oa[base + k] = ra;
      if (ob) ob[base + k] = rb;
    }
    ra += xa[k];
    rb += xb[k];
  }
}

template <class F>
hipError_t run_scan(F f, uint64_t n, uint64_t base, uint64_t *oa, uint64_t *ob, hipStream_t s) {
  // n+1 outputs; blocks cover indices 0..n inclusive
  const uint64_t nb = (n + 1 + kScanChunk - 1) / kScanChunk;
  uint64_t *sums = nullptr;
  hipError_t e = hipMallocAsync((void **)&sums, nb * 2 * sizeof(uint64_t), s);
  if (e != hipSuccess) return e;
  scan_reduce_kernel<F><<<dim3((unsigned)nb), dim3(kScanBlock), 0, s>>>(f, n, sums);
  scan_sums_kernel<<<dim3(1), dim3(kScanBlock), 0, s>>>(sums, nb);
  scan_apply_kernel<F><<<dim3((unsigned)nb), dim3(kScanBlock), 0, s>>>(f, n, sums, base, oa, ob);
  e = hipGetLastError();
  hipError_t e2 = hipFreeAsync(sums, s);
  return e != hipSuccess ? e : e2;
}

int g_cus = 0;

inline int device_cus() {
  if (g_cus == 0) {
    int dev = 0, v = 0;
    if (hipGetDevice(&dev) == hipSuccess &&
        hipDeviceGetAttribute(&v, hipDeviceAttributeMultiprocessorCount, dev) == hipSuccess && v > 0)
      g_cus = v;
    else
      g_cus = 256;
  }
  return g_cus;
}

// Persistent-style grid: at most one workgroup per CU per `per_cu`, never more
// workgroups than tiles need.
inline unsigned tile_grid(uint64_t ntiles, int waves, int per_cu) {
  const uint64_t want = (ntiles + waves - 1) / waves;
  const uint64_t cap = (uint64_t)device_cus() * per_cu;
  return (unsigned)(want < cap ? want : cap);
}

}  // namespace

hipError_t launch_decode(const DevTables &t, const uint8_t *in, const uint64_t *in_off, uint64_t in_bias,
                         uint64_t n, uint8_t *out, const uint64_t *out_off, uint64_t out_bias,
                         uint32_t *out_len, uint8_t *status, hipStream_t s) {
  if (n == 0) return hipSuccess;
  const uint64_t ntiles = (n + dec::kTileLits - 1) / dec::kTileLits;
  decode_kernel<<<dim3(tile_grid(ntiles, dec::kWaves, 1)), dim3(dec::kThreads), 0, s>>>(
      in, in_off, in_bias, n, out, out_off, out_bias, out_len, status, t.lut1, t.lut2, ntiles);
  return hipGetLastError();
}

hipError_t launch_encode_len(const DevTables &t, const uint8_t *in, const uint64_t *in_off, uint64_t in_bias,
                             uint64_t n, uint32_t *enc_len, hipStream_t s) {
  if (n == 0) return hipSuccess;
  const uint64_t ntiles = (n + enc::kTileLits - 1) / enc::kTileLits;
  encode_len_kernel<<<dim3(tile_grid(ntiles, enc::kWaves, 2)), dim3(enc::kThreads), 0, s>>>(
      in, in_off, in_bias, n, enc_len, t.len, ntiles);
  return hipGetLastError();
}

hipError_t launch_encode(const DevTables &t, const uint8_t *in, const uint64_t *in_off, uint64_t in_bias,
                         uint64_t n, uint8_t *out, const uint64_t *out_off, uint64_t out_bias, hipStream_t s) {
  if (n == 0) return hipSuccess;
  const uint64_t ntiles = (n + enc::kTileLits - 1) / enc::kTileLits;
  encode_kernel<<<dim3(tile_grid(ntiles, enc::kWaves, 1)), dim3(enc::kThreads), 0, s>>>(
      in, in_off, in_bias, n, out, out_off, out_bias, t.code, t.len, ntiles);
  return hipGetLastError();
}

hipError_t launch_offsets(const uint32_t *enc_len, uint64_t n, uint64_t base, uint64_t *out_off,
                          uint64_t *cap_off, hipStream_t s) {
  return run_scan(LenVal{enc_len}, n, base, out_off, cap_off, s);
}

hipError_t launch_capacity(const uint64_t *in_off, uint64_t n, uint64_t base, uint64_t *cap_off,
                           hipStream_t s) {
  return run_scan(CapVal{in_off}, n, base, cap_off, nullptr, s);
}

}  // namespace mhq
