// huff_encode.hip -- gfx950 batch encode of RFC 7541 Huffman literals.
//
// Semantics: HuffmanCompressor.Write + Pad (hc/huffman.go:23-37) over
// bitWriter (io/bitio.go:72-149): codes MSB-first, the last octet padded
// with 1 bits; encode_len gives ceil(sum of code lengths / 8), the size the
// Auto choice compares with the raw length (hc/io.go:172).
#include <hip/hip_runtime.h>

#include "huff_common.h"
#include "huff_kernels.h"
#include "huff_table.h"

namespace mhq {
namespace {

using namespace dev;

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
      stage_in<false, false>(ws.in_w, 0, ia - idelta, in_bytes, lane);
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
      stage_in<false, false>(ws.in_w, 0, ia - idelta, in_bytes, lane);
      zero_lds(ws.out_w, out_bytes, lane);
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

}  // namespace

hipError_t launch_encode_len(const DevTables &t, const uint8_t *in, const uint64_t *in_off, uint64_t in_bias,
                             uint64_t n, uint32_t *enc_len, hipStream_t s) {
  if (n == 0) return hipSuccess;
  const uint64_t ntiles = (n + enc::kTileLits - 1) / enc::kTileLits;
  encode_len_kernel<<<dim3(dev::tile_grid(ntiles, enc::kWaves, 2)), dim3(enc::kThreads), 0, s>>>(
      in, in_off, in_bias, n, enc_len, t.len, ntiles);
  return hipGetLastError();
}

hipError_t launch_encode(const DevTables &t, const uint8_t *in, const uint64_t *in_off, uint64_t in_bias,
                         uint64_t n, uint8_t *out, const uint64_t *out_off, uint64_t out_bias, hipStream_t s) {
  if (n == 0) return hipSuccess;
  const uint64_t ntiles = (n + enc::kTileLits - 1) / enc::kTileLits;
  encode_kernel<<<dim3(dev::tile_grid(ntiles, enc::kWaves, 1)), dim3(enc::kThreads), 0, s>>>(
      in, in_off, in_bias, n, out, out_off, out_bias, t.code, t.len, ntiles);
  return hipGetLastError();
}

}  // namespace mhq
