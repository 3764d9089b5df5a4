// huff_kernels.hip -- gfx950 (CDNA4) kernels for the RFC 7541 Huffman literal
// batch codec.  Bit-exact with minhq's hc/huffman.go + io/bitio.go (semantics
// contract: SURVEY.md §8a; restated in oracle/huff_oracle.c).
//
// Work decomposition (decode, encode, encode_len alike):
//   * a workgroup is 4 wave64s; each wave owns a tile of kLitsPerWave
//     consecutive literals;
//   * the wave stages the tile's offsets in LDS and splits the tile into 64
//     contiguous literal runs of near-equal encoded bytes (a lower_bound per
//     lane), so every lane streams one contiguous byte range in and one out;
//   * the code tables live in LDS: LUT1 (4096 x u32, two symbols per probe)
//     and LUT2 (leading-ones keyed, codes of 13..30 bits) for decode, the 256
//     code/length pairs for encode.
#include <hip/hip_runtime.h>

#include "huff_kernels.h"
#include "huff_table.h"

namespace mhq {

namespace {

constexpr int kWave = 64;
constexpr int kWavesPerBlock = 4;
constexpr int kBlock = kWave * kWavesPerBlock;
constexpr int kLitsPerWave = 512;

// ---------------------------------------------------------------------------
// Tile setup shared by all three kernels.
// ---------------------------------------------------------------------------
struct TileRun {
  uint32_t first, last;  // this lane's literal run [first, last) within the tile
  uint32_t cnt;          // literals in the tile
  uint64_t s;            // tile's first literal
};

// Loads off[s .. s+cnt] into `lds` (cnt+1 entries).  Caller synchronises.
__device__ inline void load_tile_offsets(const uint64_t *__restrict__ off, uint64_t s, uint32_t cnt,
                                         uint64_t *lds, int lane) {
  for (uint32_t j = lane; j <= cnt; j += kWave) lds[j] = off[s + j];
}

// First index j in [0, cnt) with lds[j] >= target, or cnt.
__device__ inline uint32_t lower_bound_lds(const uint64_t *lds, uint32_t cnt, uint64_t target) {
  uint32_t lo = 0, hi = cnt;
  while (lo < hi) {
    uint32_t mid = (lo + hi) >> 1;
    if (lds[mid] < target) lo = mid + 1;
    else hi = mid;
  }
  return lo;
}

// Byte-balanced split of the tile into 64 contiguous literal runs.
__device__ inline void split_runs(const uint64_t *lds_in, uint32_t cnt, int lane, TileRun &r) {
  const uint64_t b0 = lds_in[0];
  const uint64_t total = lds_in[cnt] - b0;
  const uint64_t t0 = b0 + (total * (uint64_t)lane) / kWave;
  const uint64_t t1 = b0 + (total * (uint64_t)(lane + 1)) / kWave;
  r.first = lane == 0 ? 0u : lower_bound_lds(lds_in, cnt, t0);
  r.last = lane == kWave - 1 ? cnt : lower_bound_lds(lds_in, cnt, t1);
}

// ---------------------------------------------------------------------------
// Word-granular reader over a tile's input bytes.  Words are fetched aligned
// and byte-swapped so bit 31 is the first bit of the stream (MSB-first, as
// io/bitio.go:202-214 reads it).  Fetches past the tile's last byte are
// clamped to the last in-range word: those bits are never used for a decision
// (see decode_lane).
// ---------------------------------------------------------------------------
struct WordReader {
  const uint32_t *base;  // 4-byte aligned
  uint64_t lastw;        // index of the last word holding a tile byte
  __device__ inline uint32_t word(uint64_t k) const {
    k = k < lastw ? k : lastw;
    return __builtin_bswap32(__builtin_nontemporal_load(base + k));
  }
  // 32 stream bits starting at bit position bp.
  __device__ inline uint32_t window(uint64_t bp) const {
    const uint64_t k = bp >> 5;
    const uint32_t sh = (uint32_t)bp & 31u;
    const uint32_t a = word(k);
    const uint32_t b = word(k + 1);
    return sh ? (a << sh) | (b >> (32u - sh)) : a;
  }
};

__device__ inline WordReader make_reader(const uint8_t *in, uint64_t start, uint64_t end) {
  WordReader r;
  const uintptr_t a0 = (uintptr_t)(in + start) & ~(uintptr_t)3;
  r.base = (const uint32_t *)a0;
  const uintptr_t last_byte = (uintptr_t)(in + (end > start ? end - 1 : start));
  r.lastw = (uint64_t)((last_byte - a0) >> 2);
  return r;
}

// ---------------------------------------------------------------------------
// Decode: hc/huffman.go:102-121 (+ ReadFull loop semantics, hc/io.go:92-96).
// ---------------------------------------------------------------------------
struct DecodeSmem {
  uint32_t lut1[kLut1Size];
  uint16_t lut2[kLut2Size];
  uint64_t in_off[kWavesPerBlock][kLitsPerWave + 1];
  uint64_t out_off[kWavesPerBlock][kLitsPerWave + 1];
};

__global__ __launch_bounds__(kBlock) void decode_kernel(
    const uint8_t *__restrict__ in, const uint64_t *__restrict__ in_off, uint64_t in_bias, uint64_t n,
    uint8_t *__restrict__ out, const uint64_t *__restrict__ out_off, uint64_t out_bias,
    uint32_t *__restrict__ out_len, uint8_t *__restrict__ status, const uint32_t *__restrict__ g_lut1,
    const uint16_t *__restrict__ g_lut2) {
  __shared__ DecodeSmem sm;
  const int tid = threadIdx.x;
  const int wave = tid / kWave;
  const int lane = tid % kWave;

  for (int i = tid; i < kLut1Size; i += kBlock) sm.lut1[i] = g_lut1[i];
  for (int i = tid; i < kLut2Size; i += kBlock) sm.lut2[i] = g_lut2[i];

  const uint64_t s = ((uint64_t)blockIdx.x * kWavesPerBlock + wave) * kLitsPerWave;
  const uint32_t cnt = s < n ? (uint32_t)min((uint64_t)kLitsPerWave, n - s) : 0u;
  if (cnt) {
    load_tile_offsets(in_off, s, cnt, sm.in_off[wave], lane);
    load_tile_offsets(out_off, s, cnt, sm.out_off[wave], lane);
  }
  __syncthreads();
  if (!cnt) return;

  const uint64_t *lin = sm.in_off[wave];
  const uint64_t *lout = sm.out_off[wave];
  TileRun run;
  split_runs(lin, cnt, lane, run);

  const uint64_t tile_start = lin[0] - in_bias;
  const uint64_t tile_end = lin[cnt] - in_bias;
  const WordReader rd = make_reader(in, tile_start, tile_end);
  const uint64_t bit0 = ((uintptr_t)(in + tile_start) & 3u) * 8u;  // bit offset of tile start in word 0

  for (uint32_t j = run.first; j < run.last; j++) {
    uint64_t bp = bit0 + (lin[j] - lin[0]) * 8u;
    const uint64_t endbit = bit0 + (lin[j + 1] - lin[0]) * 8u;
    uint8_t *dst = out + (lout[j] - out_bias);
    const uint64_t cap = lout[j + 1] - lout[j];
    uint64_t cnt_out = 0;
    uint8_t st = 0;
    while (cnt_out < cap) {
      const uint64_t rem = endbit - bp;
      if (rem == 0) break;  // io.EOF at a symbol boundary
      const uint32_t w = rd.window(bp);
      const uint32_t e = sm.lut1[w >> (32 - kLut1Bits)];
      const uint32_t nsym = e >> 26;
      if (nsym == 0) {
        // Long code (> 12 bits) or the all-ones EOS prefix.
        const uint32_t nw = ~w;
        const uint32_t c = nw ? (uint32_t)__builtin_clz(nw) : 32u;  // leading ones
        if (c >= (uint32_t)kEosOnes) {
          // 30 ones reach the childless node (hc/huffman.go:63-76): one more
          // bit is a nil child -> "invalid Huffman coding"; otherwise EOF.
          if (rem > (uint64_t)kEosOnes) st = 1;
          break;
        }
        const uint32_t sub = (w << (c + 1)) >> (32 - kLut2SubBits);
        const uint32_t e2 = sm.lut2[(c << kLut2SubBits) | sub];
        const uint32_t L = e2 >> 8;
        if (L == 0 || L > rem) break;  // partial code at the end: dropped
        dst[cnt_out++] = (uint8_t)(e2 & 0xffu);
        bp += L;
        continue;
      }
      const uint32_t len0 = (e >> 16) & 31u;
      const uint32_t tot = (e >> 21) & 31u;
      if (len0 > rem) break;  // partial code: dropped silently
      dst[cnt_out++] = (uint8_t)(e & 0xffu);
      if (nsym == 2 && tot <= rem && cnt_out < cap) {
        dst[cnt_out++] = (uint8_t)((e >> 8) & 0xffu);
        bp += tot;
      } else {
        bp += len0;
      }
    }
    out_len[s + j] = (uint32_t)cnt_out;
    status[s + j] = st;
  }
}

// ---------------------------------------------------------------------------
// Encode length: sum of code lengths per literal -> bytes (hc/huffman.go:23-37
// + Pad).  This is also the input to the Auto decision (hc/io.go:172).
// ---------------------------------------------------------------------------
struct EncodeSmem {
  uint32_t code[256];
  uint32_t len[256];
  uint64_t in_off[kWavesPerBlock][kLitsPerWave + 1];
  uint64_t out_off[kWavesPerBlock][kLitsPerWave + 1];
};

__global__ __launch_bounds__(kBlock) void encode_len_kernel(
    const uint8_t *__restrict__ in, const uint64_t *__restrict__ in_off, uint64_t in_bias, uint64_t n,
    uint32_t *__restrict__ enc_len, const uint8_t *__restrict__ g_len) {
  __shared__ EncodeSmem sm;
  const int tid = threadIdx.x;
  const int wave = tid / kWave;
  const int lane = tid % kWave;
  for (int i = tid; i < 256; i += kBlock) sm.len[i] = g_len[i];
  const uint64_t s = ((uint64_t)blockIdx.x * kWavesPerBlock + wave) * kLitsPerWave;
  const uint32_t cnt = s < n ? (uint32_t)min((uint64_t)kLitsPerWave, n - s) : 0u;
  if (cnt) load_tile_offsets(in_off, s, cnt, sm.in_off[wave], lane);
  __syncthreads();
  if (!cnt) return;
  const uint64_t *lin = sm.in_off[wave];
  TileRun run;
  split_runs(lin, cnt, lane, run);
  for (uint32_t j = run.first; j < run.last; j++) {
    const uint8_t *p = in + (lin[j] - in_bias);
    const uint64_t L = lin[j + 1] - lin[j];
    uint64_t bits = 0;
    uint64_t i = 0;
    // head bytes up to a 4-byte boundary, then whole words, then the tail
    for (; i < L && (((uintptr_t)(p + i)) & 3u); i++) bits += sm.len[p[i]];
    for (; i + 4 <= L; i += 4) {
      const uint32_t w = *(const uint32_t *)(p + i);
      bits += sm.len[w & 0xffu] + sm.len[(w >> 8) & 0xffu] + sm.len[(w >> 16) & 0xffu] + sm.len[w >> 24];
    }
    for (; i < L; i++) bits += sm.len[p[i]];
    enc_len[s + j] = (uint32_t)((bits + 7u) >> 3);
  }
}

// ---------------------------------------------------------------------------
// Encode: concatenated codes MSB-first, then Pad(0xff) (hc/huffman.go:23-37,
// io/bitio.go:72-149).
// ---------------------------------------------------------------------------
__global__ __launch_bounds__(kBlock) void encode_kernel(
    const uint8_t *__restrict__ in, const uint64_t *__restrict__ in_off, uint64_t in_bias, uint64_t n,
    uint8_t *__restrict__ out, const uint64_t *__restrict__ out_off, uint64_t out_bias,
    const uint32_t *__restrict__ g_code, const uint8_t *__restrict__ g_len) {
  __shared__ EncodeSmem sm;
  const int tid = threadIdx.x;
  const int wave = tid / kWave;
  const int lane = tid % kWave;
  for (int i = tid; i < 256; i += kBlock) {
    sm.code[i] = g_code[i];
    sm.len[i] = g_len[i];
  }
  const uint64_t s = ((uint64_t)blockIdx.x * kWavesPerBlock + wave) * kLitsPerWave;
  const uint32_t cnt = s < n ? (uint32_t)min((uint64_t)kLitsPerWave, n - s) : 0u;
  if (cnt) {
    load_tile_offsets(in_off, s, cnt, sm.in_off[wave], lane);
    load_tile_offsets(out_off, s, cnt, sm.out_off[wave], lane);
  }
  __syncthreads();
  if (!cnt) return;
  const uint64_t *lin = sm.in_off[wave];
  const uint64_t *lout = sm.out_off[wave];
  TileRun run;
  split_runs(lin, cnt, lane, run);
  for (uint32_t j = run.first; j < run.last; j++) {
    const uint8_t *p = in + (lin[j] - in_bias);
    const uint64_t L = lin[j + 1] - lin[j];
    uint8_t *dst = out + (lout[j] - out_bias);
    const uint64_t cap = lout[j + 1] - lout[j];
    uint64_t acc = 0;
    uint32_t nacc = 0;
    uint64_t o = 0;
    for (uint64_t i = 0; i < L; i++) {
      const uint32_t b = p[i];
      acc = (acc << sm.len[b]) | sm.code[b];
      nacc += sm.len[b];
      while (nacc >= 8) {
        nacc -= 8;
        if (o < cap) dst[o] = (uint8_t)(acc >> nacc);
        o++;
      }
    }
    if (nacc) {  // Pad(0xff): the top 8-nacc bits of 0xff
      const uint32_t padn = 8 - nacc;
      if (o < cap) dst[o] = (uint8_t)((acc << padn) | ((1u << padn) - 1u));
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

inline unsigned tiles_grid(uint64_t n) {
  const uint64_t waves = (n + kLitsPerWave - 1) / kLitsPerWave;
  return (unsigned)((waves + kWavesPerBlock - 1) / kWavesPerBlock);
}

}  // namespace

hipError_t launch_decode(const DevTables &t, const uint8_t *in, const uint64_t *in_off, uint64_t in_bias,
                         uint64_t n, uint8_t *out, const uint64_t *out_off, uint64_t out_bias,
                         uint32_t *out_len, uint8_t *status, hipStream_t s) {
  if (n == 0) return hipSuccess;
  decode_kernel<<<dim3(tiles_grid(n)), dim3(kBlock), 0, s>>>(in, in_off, in_bias, n, out, out_off, out_bias,
                                                            out_len, status, t.lut1, t.lut2);
  return hipGetLastError();
}

hipError_t launch_encode_len(const DevTables &t, const uint8_t *in, const uint64_t *in_off, uint64_t in_bias,
                             uint64_t n, uint32_t *enc_len, hipStream_t s) {
  if (n == 0) return hipSuccess;
  encode_len_kernel<<<dim3(tiles_grid(n)), dim3(kBlock), 0, s>>>(in, in_off, in_bias, n, enc_len, t.len);
  return hipGetLastError();
}

hipError_t launch_encode(const DevTables &t, const uint8_t *in, const uint64_t *in_off, uint64_t in_bias,
                         uint64_t n, uint8_t *out, const uint64_t *out_off, uint64_t out_bias, hipStream_t s) {
  if (n == 0) return hipSuccess;
  encode_kernel<<<dim3(tiles_grid(n)), dim3(kBlock), 0, s>>>(in, in_off, in_bias, n, out, out_off, out_bias,
                                                            t.code, t.len);
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
